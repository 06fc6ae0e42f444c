# round 5 dd: same-box A/B of the linear-DMA wait position (HM_FFM_LIN_DEFER 1 / 0), interleaved
set -o pipefail
mkdir -p gpurun_out/r5
for d in 1 0 1 0 1 0; do
  HM_FFM_LIN_DEFER=$d timeout -k 10 200 python -u bench.py > gpurun_out/r5/bench_lin_$d.log 2>&1
  rc=$?; echo "lin_defer=$d rc=$rc $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*' gpurun_out/r5/bench_lin_$d.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
