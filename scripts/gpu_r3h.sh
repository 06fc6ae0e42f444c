#!/bin/bash
# Round 3: pad-slot writes moved off the FTRL wave in the bf16 pipeline; default bench x2,
# fp32 sg register kernel (variant 5) once, FFM GPU tests.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r3h_pytest_ffm.log
timeout -k 10 200 python bench.py 2>&1 | tee gpurun_out/r3h_bench_1.log
timeout -k 10 200 python bench.py 2>&1 | tee gpurun_out/r3h_bench_2.log
HM_FFM_VARIANT=5 timeout -k 10 200 python bench.py --state fp32 --fp32-run 0 2>&1 | tee gpurun_out/r3h_bench_reg.log
