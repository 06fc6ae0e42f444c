#!/bin/bash
# Round 3: hot-feature pre-aggregation defaults — linear GPU tests + linear_hashed bench config.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_linear.py -m gpu -x -v --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r3o_pytest_linear.log
timeout -k 10 300 python benchmarks/bench_configs.py linear_hashed 2>&1 | tee gpurun_out/r3o_linear_hashed.log
HM_LINEAR_HOT=0 timeout -k 10 300 python benchmarks/bench_configs.py linear_hashed 2>&1 | tee gpurun_out/r3o_linear_hashed_nohot.log
