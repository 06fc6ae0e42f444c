# round 5 ac: train_fm waves per workgroup (1 / 2 / 4) at the 128-workgroup default: config-2 rate and parity
set -o pipefail
mkdir -p gpurun_out/r5
export HM_NO_AUTOBUILD=1
for wpb in 1 4 2 1 4 2; do
  HM_FM_WPB=$wpb timeout -k 10 200 python -u benchmarks/bench_configs.py fm > gpurun_out/r5/fm_wpb_$wpb.log 2>&1
  rc=$?; echo "wpb=$wpb rc=$rc $(grep -o '"rows_per_s": [0-9.]*\|"heldout_logloss_after_2_epochs": [0-9.]*' gpurun_out/r5/fm_wpb_$wpb.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
for wpb in 1 4; do
  HM_FM_WPB=$wpb PROBE_REPS=3 timeout -k 10 400 python -u benchmarks/fm_grid_parity_probe.py 128 > gpurun_out/r5/fm_wpb_parity_$wpb.jsonl 2>/dev/null
  rc=$?; echo "parity wpb=$wpb rc=$rc"; cat gpurun_out/r5/fm_wpb_parity_$wpb.jsonl; [ $rc -eq 0 ] || exit $rc
done
