#!/bin/bash
# round 6 validation (final tree candidates): whole GPU suite twice (Hogwild-bound tests differ run
# to run), smoke, the driver's bench x2, the default bench
set -o pipefail
O=gpurun_out/r6al
mkdir -p $O
export HM_NO_AUTOBUILD=1
for rep in 1 2; do
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu_$rep.log 2>&1
grep -E "FAILED" $O/pytest_gpu_$rep.log | head -5; tail -1 $O/pytest_gpu_$rep.log
done
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
for rep in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_$rep.log 2>&1 || exit 3
tail -1 $O/bench_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d.get('logloss_gap'), d.get('value_bf16_state'), d.get('logloss_gap_bf16'))"
done
timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1 || exit 4
tail -1 $O/bench_default.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['steps'], d['value'], d.get('logloss_gap'), d.get('value_bf16_state'), d.get('logloss_gap_bf16'))"
echo ok
