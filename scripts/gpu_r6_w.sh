#!/bin/bash
# round 6: the lost-update invariant test, the bench-scale parity test, the default bench (40 / 8)
# and kernel stats of the driver's bench config with the side-table linear mode
set -o pipefail
O=gpurun_out/r6w
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -x -v --timeout 300 --timeout-method thread -k "hot_linear or bench_scale" > $O/pytest_new.log 2>&1 || { tail -30 $O/pytest_new.log; exit 1; }
tail -1 $O/pytest_new.log
timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1 || exit 2
tail -1 $O/bench_default.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default40', d['value'], d.get('logloss_gap'), d.get('value_bf16_state'), d.get('logloss_gap_bf16'))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/bench_prof.log 2>&1 || exit 3
find $O/prof -name "*kernel_stats.csv" | head -3
echo ok
