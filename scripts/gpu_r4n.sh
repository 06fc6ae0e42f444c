#!/bin/bash
# Adam / SGD / momentum parity vs rows in flight down to one wave (converging step sizes,
# 300 K rows); FFM headline logloss parity at 8 gloo ranks on one card vs one rank on the same
# total rows (the bench's shape: 2^20 features, batch 262,144, mix every 10).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4n
mkdir -p $O
export HM_NO_AUTOBUILD=1
HM_RULE_WAVES="1,2,4,8,16,32" timeout -k 10 600 python -u benchmarks/linear_rules_parity.py 300000 "-opt adam -eta0 0.01" \
  "-opt sgd -eta0 0.05" "-opt momentum -eta0 0.005" > $O/linear_fewwaves.jsonl 2>&1
HM_DIST_BACKEND=gloo timeout -k 10 1000 python -u benchmarks/dp_parity.py --worlds 8 --device cuda --steps 10 \
  --warmup 0 --batch 262144 --hash-bits 20 --eval-rows 262144 --same-steps 0 > $O/dp_parity_gloo_w8.jsonl 2>&1
