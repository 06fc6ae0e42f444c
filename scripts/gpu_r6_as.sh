#!/bin/bash
# round 6: train_fm early-training ramp on fewer XCDs (the first 2^20 rows; 200 K-row fixture), x2
set -o pipefail
O=gpurun_out/r6as
mkdir -p $O
export HM_NO_AUTOBUILD=1
for cfg in "1 128" "2 128" "1 256" "2 256" "1 128" "2 128" "1 256" "2 256"; do
  set -- $cfg
  HM_FM_RAMP_XCDS=$1 HM_FM_RAMP_GRID=$2 timeout -k 10 300 python -u -m pytest tests/test_fm.py -m gpu -s -q --timeout 300 --timeout-method thread -k "test_fm_gpu_logloss_parity and not past" > $O/early_x$1_g$2.log 2>&1
  echo "x$1 g$2 $(grep -ho "'gpu': [0-9.]*" $O/early_x$1_g$2.log | tr '\n' ' ')"
done
echo ok
