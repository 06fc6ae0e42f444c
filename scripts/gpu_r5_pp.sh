# round 5 pp: train_fm w inside each feature's V record -- FM GPU tests, same-box A/B, option sweep
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests/test_fm.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r5/pytest_fm_pp.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r5/pytest_fm_pp.log; [ $rc -eq 0 ] || exit $rc
for sep in 0 1 0 1 0 1; do
  HM_FM_W_RECORD=$((1-sep)) timeout -k 10 200 python -u benchmarks/bench_configs.py fm > gpurun_out/r5/fm_wrec_$sep.log 2>&1
  rc=$?; echo "separate=$sep rc=$rc $(grep -o '"rows_per_s": [0-9.]*\|"heldout_logloss_after_2_epochs": [0-9.]*' gpurun_out/r5/fm_wrec_$sep.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u benchmarks/fm_option_rate_sweep.py > gpurun_out/r5/fm_option_rate_sweep_wrec.jsonl 2>/dev/null
echo "sweep rc=$?"
