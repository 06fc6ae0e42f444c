#!/bin/bash
# round 6 probe (not kept): side-table flush atomics into a scratch copy (hacc lines stay in L2;
# wrong semantics, rate only) vs the real flush vs plain
set -o pipefail
O=gpurun_out/r6ab
mkdir -p $O
export HM_NO_AUTOBUILD=1
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --alt-run 0 > $O/bench_$tag.log 2>&1 || { tail -5 $O/bench_$tag.log; exit 1; }
  tail -1 $O/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d.get('logloss_gap'))"
}
run side
run scratch HM_PROBE_HFLUSH=1
run plain HM_FFM_LIN_ATOMIC=0
run side_b
run scratch_b HM_PROBE_HFLUSH=1
echo ok
