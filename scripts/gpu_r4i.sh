#!/bin/bash
# GBT with 2-statistic histograms (gbt2) vs 3; linear owner-mode hot features for every rule.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4i
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_trees.py \
  tests/test_xgboost.py > $O/pytest_trees.log 2>&1
for g in 0 1; do
  echo "== gbt2 $g" >> $O/gbdt_ab.log
  HM_GBT2=$g timeout -k 10 300 python -u benchmarks/bench_configs.py gbdt >> $O/gbdt_ab.log 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gbdt -o gbdt -- \
  python3 benchmarks/bench_configs.py gbdt > $O/prof_gbdt.log 2>&1
HM_RULE_WAVES="512,1024" timeout -k 10 900 python -u benchmarks/linear_rules_parity.py 1000000 > $O/linear_owner.jsonl 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_linear.py \
  > $O/pytest_linear.log 2>&1 || true
tail -5 $O/pytest_linear.log
