#!/bin/bash
# round 6: FM hot-feature write-through on one hot update in N (parity + config-2 rate); BPR
# three-stage pipeline (rate A/B + quality test)
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
for ev in 16 64 256; do
  HM_FM_HOT_FRAC=0.002 HM_FM_HOT_EVERY=$ev HM_BENCH_FM_OPTS="-grid 256" timeout -k 10 200 python benchmarks/bench_configs.py fm > $O/fm_rate_e${ev}_g256.log 2>&1 || exit 1
done
PROBE_HOT=0.002 PROBE_HOT_EVERY=16,64,256 PROBE_REPS=2 timeout -k 10 400 python -u benchmarks/fm_grid_parity_probe.py 256 > $O/fm_hot_every_parity.jsonl 2> $O/fm_hot_every_parity.err || exit 2
for v in 2 0 2 0; do
  HM_BPR_VARIANT=$v timeout -k 10 300 python benchmarks/bench_configs.py bprmf > $O/bpr_v$v.log 2>&1 || exit 3
  cat $O/bpr_v$v.log >> $O/bpr_ab.log
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_mf.py -k "bpr" > $O/pytest_bpr.log 2>&1 || exit 4
echo ok
