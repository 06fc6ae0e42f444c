#!/bin/bash
# round 6: the rebuilt library (comment-only source change) loads and passes: smoke, FFM GPU tests, bench
set -o pipefail
O=gpurun_out/r6bm
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u -m pytest tests/test_ffm.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_ffm.log 2>&1 || { grep FAILED $O/pytest_ffm.log | head; tail -3 $O/pytest_ffm.log; exit 2; }
tail -1 $O/pytest_ffm.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 3
cut -c1-200 $O/bench.json
echo ok
