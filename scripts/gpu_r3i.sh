#!/bin/bash
# Round 3: bf16 V in the block layout (register-prefetch ffm_sg_kernel, pads spread) vs 16-B slots.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
for rep in 1 2; do
  HM_FFM_BF16_LAYOUT=block timeout -k 10 200 python bench.py --fp32-run 0 2>&1 | tee gpurun_out/r3i_bench_block_$rep.log
  timeout -k 10 200 python bench.py --fp32-run 0 2>&1 | tee gpurun_out/r3i_bench_slot16_$rep.log
done
