#!/bin/bash
# round 6: hot features' linear (z, n) in a side table during a launch (HM_FFM_LIN_ATOMIC=4, block
# sums in LDS, atomics at block end) vs plain record stores (0); rate + gap on the driver's stream
set -o pipefail
O=gpurun_out/r6r
mkdir -p $O
export HM_NO_AUTOBUILD=1
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --alt-run 0 > $O/bench_$tag.log 2>&1 || { tail -5 $O/bench_$tag.log; exit 1; }
  tail -1 $O/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d.get('logloss_gap'))"
}
run side2k HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_HOT=2048
run plain HM_FFM_LIN_ATOMIC=0
run side1k HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_HOT=1024
run side2k_b HM_FFM_LIN_ATOMIC=4 HM_FFM_LIN_HOT=2048
timeout -k 10 300 python -u -m pytest tests/test_ffm.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_ffm.log 2>&1 || { tail -15 $O/pytest_ffm.log; exit 2; }
tail -1 $O/pytest_ffm.log
echo ok
