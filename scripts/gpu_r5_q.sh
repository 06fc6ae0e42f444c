# round 5 q: FFM single-block test after bounding the deferred rows' grid, repeated 3x in one process
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest tests/test_ffm.py -m gpu -v -s --timeout 200 --timeout-method thread -k "single_block or multihot" > gpurun_out/r5/pytest_ffm_q.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5/pytest_ffm_q.log
