# round 5 z: the bench's cpu-generated criteo_ffm stream, fp32 and bf16 state held-out logloss (x2)
set -o pipefail
mkdir -p gpurun_out/r5
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --gen-device cpu --data criteo_ffm > gpurun_out/r5/bench_cpugen_$r.log 2>&1
  rc=$?; echo "rep $r rc=$rc $(grep -o '"logloss_heldout": [0-9.]*\|"logloss_heldout_bf16": [0-9.]*\|"value": [0-9.]*\|"value_bf16_state": [0-9.]*' gpurun_out/r5/bench_cpugen_$r.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
