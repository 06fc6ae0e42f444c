#!/bin/bash
# Heap-layout tree levels (no host read per level): tree tests, GBDT / XGBoost A/B, kernel trace.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4y
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_trees.py \
  tests/test_xgboost.py > $O/pytest_trees.log 2>&1
tail -2 $O/pytest_trees.log
for h in 0 1; do
  echo "== heap $h" >> $O/gbdt_ab.log
  HM_TREE_HEAP=$h timeout -k 10 300 python -u benchmarks/bench_configs.py gbdt xgboost rf >> $O/gbdt_ab.log 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gbdt -o gbdt -- \
  python3 benchmarks/bench_configs.py gbdt > $O/prof_gbdt.log 2>&1
