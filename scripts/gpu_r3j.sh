#!/bin/bash
# Round 3: bf16 V in 12-B {V | G} slots (ffm_pipe_sg12_kernel) vs 16-B slots; FFM GPU tests.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r3j_pytest_ffm.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee gpurun_out/r3j_smoke.log
for rep in 1 2; do
  timeout -k 10 200 python bench.py --fp32-run 0 2>&1 | tee gpurun_out/r3j_bench_slot12_$rep.log
  HM_FFM_BF16_LAYOUT=slot16 timeout -k 10 200 python bench.py --fp32-run 0 2>&1 | tee gpurun_out/r3j_bench_slot16_$rep.log
done
