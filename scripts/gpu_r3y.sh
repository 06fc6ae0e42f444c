#!/bin/bash
# Round 3: routing fused into the partition count when every row is active (trees.hip
# route_count_kernel): tree / xgboost GPU tests, then GBDT / XGBoost / RF configs twice.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 500 python -u -m pytest tests/test_trees.py tests/test_xgboost.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3y_pytest_trees.log 2>&1
tail -2 gpurun_out/r3y_pytest_trees.log
for rep in 1 2; do
  timeout -k 10 300 python -u benchmarks/bench_configs.py gbdt xgboost rf >> gpurun_out/r3y_trees.log 2>&1
done
grep '^{' gpurun_out/r3y_trees.log | cut -c1-220
echo done
