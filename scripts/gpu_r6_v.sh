#!/bin/bash
# round 6: side-table linear mode in both pipelined kernels (fp32 sg32: 2,048 hot features, bf16
# sg12: 1,024), default grid 2,048 for side-table launches; full bench (fp32 + bf16) vs plain
set -o pipefail
O=gpurun_out/r6v
mkdir -p $O
export HM_NO_AUTOBUILD=1
run() {  # tag, args, env...
  local tag=$1; local args=$2; shift; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $args > $O/bench_$tag.log 2>&1 || { tail -5 $O/bench_$tag.log; exit 1; }
  tail -1 $O/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d.get('logloss_gap'), d.get('value_bf16_state'), d.get('logloss_gap_bf16'))"
}
run side ""
run plain "" HM_FFM_LIN_ATOMIC=0
run side_g4k "--grid 4096"
run side_b ""
timeout -k 10 300 python -u -m pytest tests/test_ffm.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_ffm.log 2>&1 || { tail -15 $O/pytest_ffm.log; exit 2; }
tail -1 $O/pytest_ffm.log
echo ok
