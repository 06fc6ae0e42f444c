#!/bin/bash
# GPU call: tree kernel tests, GBDT / RF config benchmarks with a torch profile of GBDT.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests/test_trees.py tests/test_xgboost.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_d.log 2>&1
timeout -k 10 600 python -u benchmarks/bench_configs.py gbdt rf > gpurun_out/configs_d.log 2>&1
timeout -k 10 600 python -u benchmarks/bench_configs.py gbdt --profile > gpurun_out/configs_d_prof.log 2>&1
echo done
