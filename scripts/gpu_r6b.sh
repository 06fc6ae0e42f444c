#!/bin/bash
# Trees: 2,048-block route + count pass for <= 256 keys: tests, benches.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6b
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_trees.py \
  tests/test_xgboost.py > $O/pytest_trees.log 2>&1
for rep in 1 2; do
  timeout -k 10 300 python -u benchmarks/bench_configs.py gbdt xgboost rf >> $O/trees.log 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gbdt -o gbdt -- \
  python3 benchmarks/bench_configs.py gbdt > $O/prof_gbdt.log 2>&1
