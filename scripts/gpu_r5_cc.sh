# round 5 cc: the linear-state DMA wait moved to its first use (W_LIN wave): FFM tests + bench x2
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r5/pytest_ffm_cc.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/r5/pytest_ffm_cc.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u bench.py > gpurun_out/r5/bench_cc_$r.log 2>&1
  rc=$?; echo "bench $r rc=$rc $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*\|"value_bf16_state": [0-9.]*' gpurun_out/r5/bench_cc_$r.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
