#!/bin/bash
# Fused MFMA top-k: GPU tests + bench, then the whole GPU suite, smoke and the headline bench.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_topk_mips.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_mips.log 2>&1
timeout -k 10 300 python -u benchmarks/mips_bench.py > gpurun_out/mips_bench.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_g.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_g.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_g.log 2>&1
echo done
