# round 5 ss: same-stream gap vs the sequential engine (0.44501) with the linear records
set -o pipefail
mkdir -p gpurun_out/r5
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --gen-device cpu > gpurun_out/r5/bench_cpugen_linrec_$r.log 2>&1
  rc=$?; echo "rep=$r rc=$rc $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*\|"value_bf16_state": [0-9.]*\|"logloss_heldout_bf16": [0-9.]*' gpurun_out/r5/bench_cpugen_linrec_$r.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
