# round 5 nn: what the linear (FTRL) path costs in the fp32 FFM kernel (experiment bits; timing only)
set -o pipefail
mkdir -p gpurun_out/r5
for dbg in 0 1 2 4 7 0; do
  HM_FFM_LIN_DBG=$dbg timeout -k 10 200 python -u bench.py > gpurun_out/r5/bench_lindbg_$dbg.log 2>&1
  rc=$?; echo "lin_dbg=$dbg rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r5/bench_lindbg_$dbg.log | head -1)"; [ $rc -eq 0 ] || exit $rc
done
echo "== -disable_wi"; timeout -k 10 200 python -u benchmarks/ffm_option_rate_sweep.py 2>/dev/null | head -3
