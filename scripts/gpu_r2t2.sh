#!/bin/bash
# FFM polled kernel with slot handover: grid-1 trace vs vmcnt variant, semantics probe, tests, A/B
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 300 python -u benchmarks/probes/ffm_poll_trace.py > gpurun_out/ffm_poll_trace.log 2>&1
TAG=r2z2 bash scripts/gpu_r2z.sh
