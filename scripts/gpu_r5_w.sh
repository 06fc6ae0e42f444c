# round 5 w: non-temporal V/G stores in the fp32 FFM kernel (variant 12) vs default, interleaved
set -o pipefail
mkdir -p gpurun_out/r5
for v in 0 12 0 12; do
  HM_FFM_VARIANT=$v timeout -k 10 200 python -u bench.py > gpurun_out/r5/bench_nt_$v.log 2>&1
  rc=$?; echo "v=$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5/bench_nt_$v.log) $(grep -o '"logloss_heldout": [0-9.]*' gpurun_out/r5/bench_nt_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
