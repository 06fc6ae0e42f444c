#!/bin/bash
# round 6: train_fm GPU tests with the early-training ramp (first 2^20 rows on 8 XCDs at grid 128,
# then 6 XCDs at 256), twice (Hogwild runs differ), + config-2 rate
set -o pipefail
O=gpurun_out/r6ac
mkdir -p $O
export HM_NO_AUTOBUILD=1
for rep in 1 2; do
timeout -k 10 600 python -u -m pytest tests/test_fm.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_fm_$rep.log 2>&1; rc=$?
tail -1 $O/pytest_fm_$rep.log; grep -E "^\{'sequential|FAILED" $O/pytest_fm_$rep.log | head -6
[ $rc -eq 0 ] || exit 1
done
timeout -k 10 200 python benchmarks/bench_configs.py fm > $O/fm_rate_default.log 2>&1 || exit 2
tail -1 $O/fm_rate_default.log | cut -c1-250
echo ok
