#!/bin/bash
# Linear: the Adam family and momentum at fewer rows in flight (converging step sizes), a repeat
# of every rule at 512 for run-to-run spread; the SQL statement after the UDTF argument fixes.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4m
mkdir -p $O
export HM_NO_AUTOBUILD=1
HM_RULE_WAVES="64,128,256" timeout -k 10 600 python -u benchmarks/linear_rules_parity.py 1000000 "-opt adam -eta0 0.01" \
  "-opt nadam -eta0 0.01" "-opt eve -eta0 0.01" "-opt adamhd -eta0 0.01" "-opt momentum -eta0 0.005" > $O/linear_lowwaves.jsonl 2>&1
HM_RULE_WAVES="512" timeout -k 10 600 python -u benchmarks/linear_rules_parity.py 1000000 > $O/linear_rep512.jsonl 2>&1
HM_SQL_PROFILE=1 timeout -k 10 600 python -u benchmarks/sql_ftvec_bench.py 1000000 cuda arrow > $O/sql_ftvec.log 2> $O/sql_ftvec.err
