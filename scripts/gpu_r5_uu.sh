# round 5 uu: bf16 tail-zeroing fix for 4-B record access -- explicit-field tests + LPACK=0 same-stream run
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest tests/test_ffm.py -m gpu -x -v --timeout 200 --timeout-method thread -k "explicit_fields or single_block" > gpurun_out/r5/pytest_ffm_uu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r5/pytest_ffm_uu.log; [ $rc -eq 0 ] || exit $rc
HM_FFM_LPACK=0 timeout -k 10 300 python -u bench.py --gen-device cpu > gpurun_out/r5/bench_uu.log 2>&1
rc=$?; echo "LPACK=0 rc=$rc $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*\|"value_bf16_state": [0-9.]*\|"logloss_heldout_bf16": [0-9.]*' gpurun_out/r5/bench_uu.log | tr '\n' ' ')"
