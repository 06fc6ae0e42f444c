# round 5 oo: FFM linear state as 16-B records inside the feature blocks -- full GPU suite, A/B, option sweep
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r5/pytest_gpu_oo.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r5/pytest_gpu_oo.log; [ $rc -eq 0 ] || exit $rc
for sep in 0 1 0 1 0 1; do
  HM_FFM_LIN_SEPARATE=$sep timeout -k 10 200 python -u bench.py > gpurun_out/r5/bench_linrec_$sep.log 2>&1
  rc=$?; echo "separate=$sep rc=$rc $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*\|"value_bf16_state": [0-9.]*\|"logloss_heldout_bf16": [0-9.]*' gpurun_out/r5/bench_linrec_$sep.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u benchmarks/ffm_option_rate_sweep.py > gpurun_out/r5/ffm_option_rate_sweep_linrec.jsonl 2>/dev/null
echo "sweep rc=$?"
