#!/bin/bash
# round 6 (session 2): linear FTRL steps as float atomics (HM_FFM_LIN_ATOMIC) — rate and the
# same-stream gap on the driver's N = 1 stream, interleaved A/B; then the FFM GPU tests, the whole
# GPU suite and smoke
set -o pipefail
O=gpurun_out/r6o
mkdir -p $O
export HM_NO_AUTOBUILD=1
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_atomic_$rep.log 2>&1 || exit 1
  tail -1 $O/bench_atomic_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('atomic', d['value'], d.get('logloss_gap'), d.get('logloss_gap_bf16'), d.get('value_bf16_state'))"
  HM_FFM_LIN_ATOMIC=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_plain_$rep.log 2>&1 || exit 2
  tail -1 $O/bench_plain_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('plain', d['value'], d.get('logloss_gap'), d.get('logloss_gap_bf16'), d.get('value_bf16_state'))"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -5 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 4
echo ok
