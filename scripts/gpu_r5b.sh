#!/bin/bash
# Linear shared engine at 8 rows in flight: state re-read before the update (RELOAD) on/off.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b
mkdir -p $O
export HM_NO_AUTOBUILD=1
for r in 1 0; do
  HM_LINEAR_RELOAD=$r timeout -k 10 600 python -u benchmarks/linear_rules_parity.py 1000000 "-opt adam -eta0 0.01" \
    "-opt sgd -eta0 0.05" "-opt rmsprop -eta0 0.01" > $O/reload$r.jsonl 2>&1
done
