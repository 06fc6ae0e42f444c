#!/bin/bash
# Few-wave parity margins at the test's size (200 K rows) for every rule routed to 8 rows in flight.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4v
mkdir -p $O
export HM_NO_AUTOBUILD=1
HM_RULE_WAVES="2,4,8" timeout -k 10 900 python -u benchmarks/linear_rules_parity.py 200000 "-opt sgd -eta0 0.05" \
  "-opt momentum -eta0 0.005" "-opt nesterov -eta0 0.005" "-opt rmsprop -eta0 0.01" "-opt rmspropgraves -eta0 0.001" \
  "-opt adadelta" "-opt adam -eta0 0.01" "-opt nadam -eta0 0.01" "-opt eve -eta0 0.01" "-opt adamhd -eta0 0.01" \
  > $O/fewwaves_200k.jsonl 2>&1
