#!/bin/bash
# Linear shared engine per-rule parity at converging step sizes: owner-mode hot features on/off,
# 512 / 1024 rows in flight, 1 M Criteo-shaped rows at 2^24 dims.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4k
mkdir -p $O
export HM_NO_AUTOBUILD=1
for own in 1 0; do
  HM_LINEAR_HOT_OWNER=$own HM_RULE_WAVES="512,1024" timeout -k 10 900 python -u benchmarks/linear_rules_parity.py 1000000 \
    > $O/linear_conv_owner$own.jsonl 2>&1
done
HM_SQL_PROFILE=1 timeout -k 10 600 python -u benchmarks/sql_ftvec_bench.py 1000000 cuda arrow > $O/sql_ftvec.log 2> $O/sql_ftvec.err
