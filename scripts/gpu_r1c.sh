#!/bin/bash
# GPU call: FFM + tree kernel tests, FFM packed A/B (next-row metadata prefetch), bench.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests/test_ffm.py tests/test_trees.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_c.log 2>&1
timeout -k 10 600 python -u benchmarks/ffm_layout_ab.py --states bf16 > gpurun_out/ffm_layout_ab_c.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c.log 2>&1
echo done
