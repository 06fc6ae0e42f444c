#!/bin/bash
# round 6: hashed side-table size (2^13 / 2^14 / 2^15 slots of 128 B): rate + gap, fp32 and bf16
set -o pipefail
O=gpurun_out/r6ak
mkdir -p $O
export HM_NO_AUTOBUILD=1
for hc in 13 14 15 14 15 13; do
HM_FFM_HC_LOG=$hc timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_hc$hc.log 2>&1 || { tail -5 $O/bench_hc$hc.log; exit 1; }
tail -1 $O/bench_hc$hc.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('hc$hc', d['value'], d.get('logloss_gap'), d.get('value_bf16_state'), d.get('logloss_gap_bf16'))"
done
echo ok
