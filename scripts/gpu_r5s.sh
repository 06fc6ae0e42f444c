#!/bin/bash
# bench.py on the CPU-generated criteo_ffm stream (sequential engine: 0.44501): early ramp length.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5s
mkdir -p $O
export HM_NO_AUTOBUILD=1
for r in 0 262144 524288 2097152; do
  timeout -k 10 300 python -u bench.py --gen-device cpu --alt-run 0 --ramp-rows $r > $O/bench_cpugen_ramp${r}.log 2>&1
  echo "ramp $r: $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*\|"early_ramp_warmup_steps": [0-9]*' $O/bench_cpugen_ramp${r}.log | tr '\n' ' ')" >> $O/ab.log
done
