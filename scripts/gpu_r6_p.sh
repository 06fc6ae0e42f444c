#!/bin/bash
# round 6: the linear FTRL steps without lost updates at speed — (4) hot features' steps summed in a
# per-block LDS table and flushed by atomics every R rows; (2 / 3) plain atomics on the hot / cold
# features only (where the all-atomic cost is); fp32, the driver's N = 1 stream
set -o pipefail
O=gpurun_out/r6p
mkdir -p $O
export HM_NO_AUTOBUILD=1
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --alt-run 0 > $O/bench_$tag.log 2>&1 || exit 1
  tail -1 $O/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d.get('logloss_gap'))"
}
run ht4k_f16 HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_HOT=4096 HM_FFM_LIN_FLUSH=16
run plain HM_FFM_LIN_ATOMIC=0
run ht16k_f16 HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_HOT=16384 HM_FFM_LIN_FLUSH=16
run ht4k_f8 HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_HOT=4096 HM_FFM_LIN_FLUSH=8
run ht64k_f12 HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_HOT=65536 HM_FFM_LIN_FLUSH=12
run hot4k HM_FFM_LIN_ATOMIC=2 HM_FFM_LIN_HOT=4096
run cold4k HM_FFM_LIN_ATOMIC=3 HM_FFM_LIN_HOT=4096
echo ok
