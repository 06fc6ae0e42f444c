#!/bin/bash
# round 6: train_fm early-training ramp grid (the first 2^20 rows; 200 K-row parity fixture), x2
set -o pipefail
O=gpurun_out/r6ar
mkdir -p $O
export HM_NO_AUTOBUILD=1
for g in 64 96 128 64 96 128; do
  HM_FM_RAMP_GRID=$g timeout -k 10 300 python -u -m pytest tests/test_fm.py -m gpu -s -q --timeout 300 --timeout-method thread -k "test_fm_gpu_logloss_parity and not past" > $O/early_g$g.log 2>&1
  echo "g$g $(grep -h "sequential" $O/early_g$g.log | tr '\n' ' ' | cut -c1-300)"
done
echo ok
