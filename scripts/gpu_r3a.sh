#!/bin/bash
# Round 3: first GPU contact of the per-slot-AdaGrad FFM kernel (ffm_sg_kernel): FFM GPU tests,
# smoke, then the bench (bf16 + fp32 V) and a per-element A/B, each step time-limited.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -x -v --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r3a_pytest_ffm.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee gpurun_out/r3a_smoke.log
timeout -k 10 200 python bench.py 2>&1 | tee gpurun_out/r3a_bench.log
timeout -k 10 200 python bench.py --adagrad element 2>&1 | tee gpurun_out/r3a_bench_elementwise.log
