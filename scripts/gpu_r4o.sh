#!/bin/bash
# Owner-mode hot-feature staleness: rows per wave per chunk (CH), rows before a block pushes its
# partial sums (MIN) and chunks between forced pushes (EVERY), for Adam / SGD / momentum at 512
# rows in flight; plus hot features off.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4o
mkdir -p $O
export HM_NO_AUTOBUILD=1
for cfg in "32 32 8" "8 1 1" "4 1 1" "16 4 2" "2 1 1"; do
  set -- $cfg
  echo "== ch $1 min $2 every $3" >> $O/linear_owner_sched.log
  HM_LINEAR_HOT_CH=$1 HM_LINEAR_HOT_MIN=$2 HM_LINEAR_HOT_EVERY=$3 HM_RULE_WAVES="512" timeout -k 10 600 \
    python -u benchmarks/linear_rules_parity.py 1000000 "-opt adam -eta0 0.01" "-opt sgd -eta0 0.05" \
    "-opt momentum -eta0 0.005" "-opt nesterov -eta0 0.005" >> $O/linear_owner_sched.log 2>&1
done
echo "== hot off" >> $O/linear_owner_sched.log
HM_LINEAR_HOT=0 HM_RULE_WAVES="512" timeout -k 10 600 python -u benchmarks/linear_rules_parity.py 1000000 \
  "-opt adam -eta0 0.01" "-opt sgd -eta0 0.05" "-opt momentum -eta0 0.005" "-opt nesterov -eta0 0.005" >> $O/linear_owner_sched.log 2>&1
