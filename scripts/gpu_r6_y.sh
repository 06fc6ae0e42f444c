#!/bin/bash
# round 6: train_fm GPU tests at the new default (6 XCDs, grid 256) + config-2 rate
set -o pipefail
O=gpurun_out/r6y
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests/test_fm.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_fm.log 2>&1; rc=$?
tail -3 $O/pytest_fm.log; grep -E "FAILED|Error|assert" $O/pytest_fm.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python benchmarks/bench_configs.py fm > $O/fm_rate_default.log 2>&1 || exit 2
tail -1 $O/fm_rate_default.log | cut -c1-250
echo ok
