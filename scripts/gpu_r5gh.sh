#!/bin/bash
set -e -o pipefail
./scripts/gpu_r5h.sh && ./scripts/gpu_r5g.sh
