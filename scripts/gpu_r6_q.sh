#!/bin/bash
# round 6: is the hot-table mode's cost the flush atomics dropping hot feature-block lines from L2?
# (debug: the same atomics into a 16 KB scratch; quality meaningless there, rate only)
set -o pipefail
O=gpurun_out/r6q
mkdir -p $O
export HM_NO_AUTOBUILD=1
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --alt-run 0 > $O/bench_$tag.log 2>&1 || exit 1
  tail -1 $O/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d.get('logloss_gap'))"
}
run ht4k_f16_scratch HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_HOT=4096 HM_FFM_LIN_FLUSH=16 HM_FFM_LIN_DEBUG=1
run ht4k_f16 HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_HOT=4096 HM_FFM_LIN_FLUSH=16
run ht4k_f12_scratch HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_HOT=4096 HM_FFM_LIN_FLUSH=12 HM_FFM_LIN_DEBUG=1
run ht64_f16 HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_HOT=64 HM_FFM_LIN_FLUSH=16
echo ok
