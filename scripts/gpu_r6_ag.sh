#!/bin/bash
# round 6: bf16 side-table kernel with the hot-index wait moved from phase C to after the forward
set -o pipefail
O=gpurun_out/r6ag
mkdir -p $O
export HM_NO_AUTOBUILD=1
run() {  # tag, args, env...
  local tag=$1; local args=$2; shift; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --state bf16 --alt-run 0 $args > $O/bench_$tag.log 2>&1 || { tail -5 $O/bench_$tag.log; exit 1; }
  tail -1 $O/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d.get('logloss_gap'))"
}
run side_auto ""
run side_g3k "--grid 3072"
run side_auto_b ""
timeout -k 10 600 python -u -m pytest tests/test_ffm.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_ffm.log 2>&1; rc=$?
grep FAILED $O/pytest_ffm.log | head -5; tail -1 $O/pytest_ffm.log
[ $rc -eq 0 ] || exit 2
echo ok
