# round 5 xx: k = 8 on the pipelined fp32 kernel (32-B slots, 512-thread blocks) -- FFM GPU tests, option sweep, default bench
set -o pipefail
mkdir -p gpurun_out/r5
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests/test_ffm.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r5/pytest_ffm_xx.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/r5/pytest_ffm_xx.log | tail -4; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/ffm_option_rate_sweep.py > gpurun_out/r5/ffm_option_rate_sweep_k8.jsonl 2>/dev/null
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/r5/ffm_option_rate_sweep_k8.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py > gpurun_out/r5/bench_xx.log 2>&1
rc=$?; echo "bench rc=$rc $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*\|"value_bf16_state": [0-9.]*\|"logloss_heldout_bf16": [0-9.]*' gpurun_out/r5/bench_xx.log | tr '\n' ' ')"
