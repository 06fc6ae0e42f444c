#!/bin/bash
# FFM fp32 sg32: streaming (nt) cache policy on the slot DMAs (variant 8) A/B.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5z
mkdir -p $O
export HM_NO_AUTOBUILD=1
for rep in 1 2 3; do
  for v in 0 8; do
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py --alt-run 0 --steps 40 --warmup 5 > $O/bench_v${v}_r${rep}.log 2>&1
    echo "variant $v rep $rep: $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*' $O/bench_v${v}_r${rep}.log | tr '\n' ' ')" >> $O/ab.log
  done
done
