#!/bin/bash
# round 6: the 4 GiB-table tests with the linear records in the blocks (64-bit launches must not be
# wrapped by the side-table copies), and the FFM GPU file
set -o pipefail
O=gpurun_out/r6ad
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests/test_ffm.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_ffm.log 2>&1; rc=$?
grep -E "4gib|FAILED" $O/pytest_ffm.log | head; tail -1 $O/pytest_ffm.log
[ $rc -eq 0 ] || exit 1
echo ok
