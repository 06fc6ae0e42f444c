#!/bin/bash
# round 6: side-table mode with lane-paired flushes at grids 1024 / 512 (fewer flushes per batch)
set -o pipefail
O=gpurun_out/r6u
mkdir -p $O
export HM_NO_AUTOBUILD=1
run() {  # tag, args, env...
  local tag=$1; local args=$2; shift; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --alt-run 0 $args > $O/bench_$tag.log 2>&1 || { tail -5 $O/bench_$tag.log; exit 1; }
  tail -1 $O/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d.get('logloss_gap'))"
}
run pair_g1k "--grid 1024" HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_DBG=4
run pair_g512 "--grid 512" HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_DBG=4
run plain_g1k "--grid 1024" HM_FFM_LIN_ATOMIC=0
run plain_g512 "--grid 512" HM_FFM_LIN_ATOMIC=0
run pair_g2k "--grid 2048" HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_DBG=4
run pair_g1k_b "--grid 1024" HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_DBG=4
echo ok
