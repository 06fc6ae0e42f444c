#!/bin/bash
# round 6: side table hashed by feature id (tag check on the DMA'd entry; no per-feature index
# lookup): rate + gap x2, FFM GPU tests
set -o pipefail
O=gpurun_out/r6aj
mkdir -p $O
export HM_NO_AUTOBUILD=1
for rep in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_$rep.log 2>&1 || { tail -5 $O/bench_$rep.log; exit 1; }
tail -1 $O/bench_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d.get('logloss_gap'), d.get('value_bf16_state'), d.get('logloss_gap_bf16'))"
done
timeout -k 10 600 python -u -m pytest tests/test_ffm.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_ffm.log 2>&1; rc=$?
grep FAILED $O/pytest_ffm.log | head -5; tail -1 $O/pytest_ffm.log
[ $rc -eq 0 ] || { grep -E "^E " $O/pytest_ffm.log | head -20; exit 2; }
echo ok
