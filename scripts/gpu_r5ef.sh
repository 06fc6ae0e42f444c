#!/bin/bash
set -e -o pipefail
./scripts/gpu_r5f.sh && ./scripts/gpu_r5e.sh
