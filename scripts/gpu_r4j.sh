#!/bin/bash
# GBDT after the ballot-counted route pass and the ILP leaf sums; linear Adam/SGD/momentum gap
# isolation over rows in flight (1 wave = sequential) with and without owner-mode hot features.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4j
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_trees.py \
  tests/test_xgboost.py > $O/pytest_trees.log 2>&1
timeout -k 10 300 python -u benchmarks/bench_configs.py gbdt xgboost rf > $O/gbdt.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gbdt -o gbdt -- \
  python3 benchmarks/bench_configs.py gbdt > $O/prof_gbdt.log 2>&1
for own in 1 0; do
  HM_LINEAR_HOT_OWNER=$own HM_RULE_WAVES="1,8,64,512" timeout -k 10 600 python -u benchmarks/linear_rules_parity.py 300000 \
    "-opt adam" "-opt sgd -eta0 0.05" "-opt momentum -eta0 0.05" > $O/linear_iso_owner$own.jsonl 2>&1
done
