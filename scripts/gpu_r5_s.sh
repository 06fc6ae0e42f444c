# round 5 s: train_fm config-2 rate by grid (second epoch of 2 M rows, 2^24 features)
set -o pipefail
mkdir -p gpurun_out/r5
for g in 256 128 64 256 128 64; do
  echo "== grid $g" >> gpurun_out/r5/fm_grid_rate.log
  HM_BENCH_FM_OPTS="-grid $g" timeout -k 10 200 python -u benchmarks/bench_configs.py fm >> gpurun_out/r5/fm_grid_rate.log 2>&1
  rc=$?; echo "grid $g rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
