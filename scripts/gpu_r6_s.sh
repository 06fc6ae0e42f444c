#!/bin/bash
# round 6: bisect the side-table mode's cost (1: no block-end atomics, 2: every feature cold with
# the side-table DMAs still issued, 3: both)
set -o pipefail
O=gpurun_out/r6s
mkdir -p $O
export HM_NO_AUTOBUILD=1
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --alt-run 0 > $O/bench_$tag.log 2>&1 || { tail -5 $O/bench_$tag.log; exit 1; }
  tail -1 $O/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d.get('logloss_gap'))"
}
run side HM_FFM_LIN_ATOMIC=4
run dbg1 HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_DBG=1


run plain HM_FFM_LIN_ATOMIC=0
echo ok
