#!/bin/bash
# round 6: bf16 (sg12) side-table mode vs grid (the fp32 grid moves too), plain bf16 at 2,048
set -o pipefail
O=gpurun_out/r6af
mkdir -p $O
export HM_NO_AUTOBUILD=1
run() {  # tag, args, env...
  local tag=$1; local args=$2; shift; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --state bf16 --alt-run 0 $args > $O/bench_$tag.log 2>&1 || { tail -5 $O/bench_$tag.log; exit 1; }
  tail -1 $O/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d.get('logloss_gap'))"
}
run side_g2k "--grid 2048"
run side_g4k "--grid 4096"
run side_g8k "--grid 8192"
run plain_g2k "--grid 2048" HM_FFM_LIN_ATOMIC=0
run plain_auto "" HM_FFM_LIN_ATOMIC=0
run side_g3k "--grid 3072"
echo ok
