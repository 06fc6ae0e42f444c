#!/bin/bash
# XGBoost fused (g, h) statistics kernel: tree/xgboost GPU tests, xgboost + GBDT configs
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 400 python -u -m pytest tests/test_xgboost.py tests/test_trees.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_trees_r2aw.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_trees_r2aw.log
grep -q "Fatal\|core dumped\|Timeout\|rc=" gpurun_out/pytest_trees_r2aw.log && exit 3
timeout -k 10 400 python -u benchmarks/bench_configs.py xgboost gbdt > gpurun_out/configs_r2aw.log 2>&1
echo done
