#!/bin/bash
# round 6: train_fm with its waves confined to 1 / 2 / 4 XCDs (parity vs the 8-mapper average and
# the config-2 rate), at grids of 128 / 256 / 512 workgroups
set -o pipefail
O=gpurun_out/r6l
mkdir -p $O
export HM_NO_AUTOBUILD=1
for x in 1 2 4; do for g in 128 256 512; do
  HM_FM_XCDS=$x HM_BENCH_FM_OPTS="-grid $g" timeout -k 10 200 python benchmarks/bench_configs.py fm > $O/fm_rate_x${x}_g${g}.log 2>&1 || exit 1
done; done
PROBE_XCDS=1,2,4 PROBE_REPS=1 timeout -k 10 500 python -u benchmarks/fm_grid_parity_probe.py 128 256 512 > $O/fm_xcd_parity.jsonl 2> $O/fm_xcd_parity.err || exit 2
echo ok
