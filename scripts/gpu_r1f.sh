#!/bin/bash
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests/test_ffm.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_f.log 2>&1
timeout -k 10 600 python -u benchmarks/ffm_layout_ab.py --states bf16 --layouts packed > gpurun_out/ffm_layout_ab_f.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_f.log 2>&1
echo done
