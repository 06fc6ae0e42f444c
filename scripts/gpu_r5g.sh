#!/bin/bash
# FFM fp32 early-training gap: atomic-update kernel for the first R rows (HM_FFM_RAMP_VARIANT),
# G-only atomics (variant 7) throughput.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5g
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u benchmarks/ffm_early_parity.py 500000 v6:32768 v6:131072 v6:262144 v7:500000 \
  > $O/early_ramp_atomic.jsonl 2> $O/early.err
timeout -k 10 600 python -u benchmarks/ffm_early_parity.py 2000000 0 v6:131072 v6:500000 \
  > $O/early_ramp_atomic_2m.jsonl 2>> $O/early.err
for v in 0 7; do
  HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py --alt-run 0 --steps 20 --warmup 3 > $O/bench_v${v}.log 2>&1
  echo "variant $v: $(tail -1 $O/bench_v${v}.log | cut -c1-200)" >> $O/ab.log
done
