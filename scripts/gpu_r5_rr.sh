# round 5 rr: counters of the headline kernel with the in-block linear records, then a grid sweep
set -o pipefail
mkdir -p gpurun_out/r5
bash scripts/gpu_r5_pmc.sh > gpurun_out/r5/pmc_rr.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/r5/pmc_rr.log; exit 1; }
echo "pmc ok"
for g in 4096 8192 16384 32768 8192 2048; do
  timeout -k 10 200 python -u bench.py --grid $g > gpurun_out/r5/bench_grid_$g.log 2>&1
  rc=$?; echo "grid=$g rc=$rc $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*\|"value_bf16_state": [0-9.]*\|"logloss_heldout_bf16": [0-9.]*' gpurun_out/r5/bench_grid_$g.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
