# round 5 ah: spread of the pinned same-stream gap (bench.py --gen-device cpu) on one more box
set -o pipefail
mkdir -p gpurun_out/r5
export HM_NO_AUTOBUILD=1
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gen-device cpu > gpurun_out/r5/bench_ah.log 2>&1
  rc=$?; echo "rep=$r rc=$rc $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*\|"logloss_heldout_bf16": [0-9.]*' gpurun_out/r5/bench_ah.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
