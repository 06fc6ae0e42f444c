#!/bin/bash
# Round 2 call t: XGBoost missing directions + sharded BPR on the GPU, tree suite.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2t}"
timeout -k 10 600 python -u -m pytest tests/test_trees.py tests/test_xgboost.py tests/test_sharded.py tests/test_mf.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_$TAG.log
grep -q "Fatal\|core dumped\|Timeout" gpurun_out/pytest_$TAG.log && exit 3
timeout -k 10 600 python -u benchmarks/bench_configs.py gbdt rf > gpurun_out/configs_trees_$TAG.log 2>&1
echo done
