#!/bin/bash
# FFM fp32: all-atomic slot updates (HM_FFM_VARIANT=6) — early-training gap and throughput.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5f
mkdir -p $O
export HM_NO_AUTOBUILD=1
HM_FFM_VARIANT=6 timeout -k 10 600 python -u benchmarks/ffm_early_parity.py 500000 8 0 > $O/early_atomic.jsonl 2> $O/early_atomic.err
for rep in 1 2; do
  for v in 0 6; do
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py --alt-run 0 --steps 20 --warmup 3 > $O/bench_v${v}_r${rep}.log 2>&1
    echo "variant $v rep $rep: $(tail -1 $O/bench_v${v}_r${rep}.log | cut -c1-400)" >> $O/ab.log
  done
done
