#!/bin/bash
# Round 3: per-slot AdaGrad kernels (bf16 16-B slots via the LDS-DMA pipeline, fp32 block layout
# via ffm_sg_kernel): FFM GPU tests, bench A/B, then rocprofv3 counters of the fp32 sg kernel.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r3c_pytest_ffm.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee gpurun_out/r3c_smoke.log
timeout -k 10 200 python bench.py 2>&1 | tee gpurun_out/r3c_bench.log
timeout -k 10 200 python bench.py --adagrad element --fp32-run 0 2>&1 | tee gpurun_out/r3c_bench_elementwise.log
timeout -k 10 200 python bench.py 2>&1 | tee gpurun_out/r3c_bench_rep2.log
OUT=ffm_pmc_sg32 PAT=ffm_sg_kernel FP32=1 bash scripts/ffm_counters.sh
