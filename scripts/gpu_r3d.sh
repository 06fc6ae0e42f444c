#!/bin/bash
# Round 3: fp32 ffm_sg_kernel at 4 waves/SIMD (own V read back from the LDS image, ext-vector
# prefetch registers): GPU tests, bench (default), variant 4 (512-thread blocks) A/B, counters.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r3d_pytest_ffm.log
timeout -k 10 200 python bench.py 2>&1 | tee gpurun_out/r3d_bench.log
HM_FFM_VARIANT=4 timeout -k 10 200 python bench.py --state fp32 --fp32-run 0 2>&1 | tee gpurun_out/r3d_bench_fp32_512.log
timeout -k 10 200 python bench.py 2>&1 | tee gpurun_out/r3d_bench_rep2.log
OUT=ffm_pmc_sg32b PAT=ffm_sg_kernel FP32=1 bash scripts/ffm_counters.sh
