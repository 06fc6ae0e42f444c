#!/bin/bash
# round 6 (session 2): re-validate the tree (GPU suite, smoke, default bench), then train_fm on
# 6 / 7 of the 8 XCDs at grids 256-384 (config-2 rate + parity vs the 8-mapper average)
set -o pipefail
O=gpurun_out/r6n
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit 3
tail -1 $O/bench.log | cut -c1-200
for x in 6 7; do for g in 256 320 384; do
  HM_FM_XCDS=$x HM_BENCH_FM_OPTS="-grid $g" timeout -k 10 200 python benchmarks/bench_configs.py fm > $O/fm_rate_x${x}_g${g}.log 2>&1 || exit 4
done; done
PROBE_XCDS=6,7 PROBE_REPS=2 timeout -k 10 600 python -u benchmarks/fm_grid_parity_probe.py 256 320 384 > $O/fm_xcd_parity.jsonl 2> $O/fm_xcd_parity.err || exit 5
echo ok
