# round 5 ee: bf16 (sg12) kernel with the deferred linear-DMA wait: FFM tests, same-box A/B
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r5/pytest_ffm_ee.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/r5/pytest_ffm_ee.log; [ $rc -eq 0 ] || exit $rc
for d in 1 0 1 0 1 0; do
  HM_FFM_LIN_DEFER=$d timeout -k 10 200 python -u bench.py > gpurun_out/r5/bench_lin12_$d.log 2>&1
  rc=$?; echo "lin_defer=$d rc=$rc $(grep -o '"value": [0-9.]*\|"value_bf16_state": [0-9.]*\|"logloss_heldout_bf16": [0-9.]*' gpurun_out/r5/bench_lin12_$d.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
