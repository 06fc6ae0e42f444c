#!/bin/bash
# bench.py: the learner's early-training ramp inside the warmup (default) vs off, held-out logloss.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5r
mkdir -p $O
export HM_NO_AUTOBUILD=1
for rep in 1 2; do
  for r in 0 262144; do
    timeout -k 10 300 python -u bench.py --alt-run 0 --ramp-rows $r > $O/bench_ramp${r}_r${rep}.log 2>&1
    echo "ramp $r rep $rep: $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*\|"early_ramp_warmup_steps": [0-9]*' $O/bench_ramp${r}_r${rep}.log | tr '\n' ' ')" >> $O/ab.log
  done
done
timeout -k 10 300 python -u bench.py --gen-device cpu --data criteo_like --alt-run 0 > $O/bench_cpugen_criteo_like.log 2>&1
echo "criteo_like cpu-gen (ramp default): $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*' $O/bench_cpugen_criteo_like.log | tr '\n' ' ')" >> $O/ab.log
