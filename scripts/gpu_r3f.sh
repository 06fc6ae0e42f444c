#!/bin/bash
# Round 3: fp32 per-slot LDS-DMA pipeline (ffm_pipe_sg32_kernel) vs the register-prefetch
# ffm_sg_kernel (variant 5), same box, interleaved.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r3g_pytest_ffm.log
for rep in 1 2; do  # distributed pad writes
  timeout -k 10 200 python bench.py --state fp32 --fp32-run 0 2>&1 | tee gpurun_out/r3g_bench_pipe_$rep.log
  HM_FFM_VARIANT=5 timeout -k 10 200 python bench.py --state fp32 --fp32-run 0 2>&1 | tee gpurun_out/r3g_bench_reg_$rep.log
done
