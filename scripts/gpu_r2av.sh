#!/bin/bash
# XGBoost config on 11M HIGGS-shaped rows (GPU), plus its GPU tests
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 300 python -u -m pytest tests/test_xgboost.py -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_xgb_r2av.log 2>&1
timeout -k 10 400 python -u benchmarks/bench_configs.py xgboost > gpurun_out/configs_xgb_r2av.log 2>&1
echo done
