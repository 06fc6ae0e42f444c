# round 5 yy: train_fm grid vs parity (8-mapper average) and config-2 rate, grids 160 / 192 / 224
set -o pipefail
mkdir -p gpurun_out/r5
export HM_NO_AUTOBUILD=1
PROBE_REPS=3 timeout -k 10 500 python -u benchmarks/fm_grid_parity_probe.py 160 192 224 > gpurun_out/r5/fm_grid_parity_yy.jsonl 2> gpurun_out/r5/fm_grid_parity_yy.err
rc=$?; echo "probe rc=$rc"; cat gpurun_out/r5/fm_grid_parity_yy.jsonl; [ $rc -eq 0 ] || exit $rc
for g in 160 192 224 256; do
  HM_BENCH_FM_OPTS="-grid $g" timeout -k 10 200 python -u benchmarks/bench_configs.py fm > gpurun_out/r5/fm_grid_rate_$g.log 2>&1
  rc=$?; echo "grid=$g rc=$rc $(grep -o '"rows_per_s": [0-9.]*\|"heldout_logloss_after_2_epochs": [0-9.]*' gpurun_out/r5/fm_grid_rate_$g.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
