#!/bin/bash
# round 6: -factors 8 with the side-table linear mode (one 512-thread block per CU either way):
# rate + held-out vs the plain stores; FFM GPU tests
set -o pipefail
O=gpurun_out/r6an
mkdir -p $O
export HM_NO_AUTOBUILD=1
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --factors 8 --alt-run 0 > $O/bench_$tag.log 2>&1 || { tail -5 $O/bench_$tag.log; exit 1; }
  tail -1 $O/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d.get('logloss_heldout'), d.get('logloss_gap'))"
}
run side
run plain HM_FFM_LIN_ATOMIC=0
run side_b
run plain_b HM_FFM_LIN_ATOMIC=0
timeout -k 10 600 python -u -m pytest tests/test_ffm.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_ffm.log 2>&1; rc=$?
grep FAILED $O/pytest_ffm.log | head -5; tail -1 $O/pytest_ffm.log
[ $rc -eq 0 ] || exit 2
echo ok
