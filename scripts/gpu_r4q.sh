#!/bin/bash
# Owner-mode hot features actually on for the default -reg (rda) of every non-AdaGrad rule:
# every rule at 512 / 1024 rows in flight, two runs; owner flush schedules for three rules.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4q
mkdir -p $O
export HM_NO_AUTOBUILD=1
for rep in 1 2; do
  HM_RULE_WAVES="512,1024" timeout -k 10 900 python -u benchmarks/linear_rules_parity.py 1000000 > $O/linear_owner_rep$rep.jsonl 2>&1
done
for cfg in "8 1 1" "4 1 1"; do
  set -- $cfg
  echo "== ch $1 min $2 every $3" >> $O/linear_owner_sched.log
  HM_LINEAR_HOT_CH=$1 HM_LINEAR_HOT_MIN=$2 HM_LINEAR_HOT_EVERY=$3 HM_RULE_WAVES="512" timeout -k 10 600 \
    python -u benchmarks/linear_rules_parity.py 1000000 "-opt adam -eta0 0.01" "-opt sgd -eta0 0.05" \
    "-opt momentum -eta0 0.005" >> $O/linear_owner_sched.log 2>&1
done
