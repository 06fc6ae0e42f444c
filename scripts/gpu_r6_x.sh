#!/bin/bash
# round 6: train_fm on 6 / 7 of the 8 XCDs at grids 256-384 (config-2 rate + parity vs the
# 8-mapper average), the 8-XCD grid-128 default beside them
set -o pipefail
O=gpurun_out/r6x
mkdir -p $O
export HM_NO_AUTOBUILD=1
for x in 6 7; do for g in 256 320 384; do
  HM_FM_XCDS=$x HM_BENCH_FM_OPTS="-grid $g" timeout -k 10 200 python benchmarks/bench_configs.py fm > $O/fm_rate_x${x}_g${g}.log 2>&1 || exit 1
  echo "x$x g$g $(tail -1 $O/fm_rate_x${x}_g${g}.log | cut -c1-160)"
done; done
HM_BENCH_FM_OPTS="-grid 128" timeout -k 10 200 python benchmarks/bench_configs.py fm > $O/fm_rate_x8_g128.log 2>&1 || exit 1
echo "x8 g128 $(tail -1 $O/fm_rate_x8_g128.log | cut -c1-160)"
PROBE_XCDS=6,7 PROBE_REPS=2 timeout -k 10 700 python -u benchmarks/fm_grid_parity_probe.py 256 320 384 > $O/fm_xcd_parity.jsonl 2> $O/fm_xcd_parity.err || exit 2
cat $O/fm_xcd_parity.jsonl | cut -c1-220
echo ok
