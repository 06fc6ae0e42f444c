# round 5 aa: train_fm hot-feature shards -- tests, parity by grid (hot on / off), config-2 rate
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest tests/test_fm.py -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/r5/pytest_fm_aa.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r5/pytest_fm_aa.log; [ $rc -le 1 ] || exit $rc
PROBE_REPS=2 timeout -k 10 300 python -u benchmarks/fm_grid_parity_probe.py 256 128 > gpurun_out/r5/fm_hot_shards_parity.jsonl 2> gpurun_out/r5/fm_hot_shards_parity.err
echo "parity rc=$?"
for hot in 32 0 32 0; do
  echo "== HM_FM_HOT=$hot" >> gpurun_out/r5/fm_hot_shards_rate.log
  HM_FM_HOT=$hot timeout -k 10 200 python -u benchmarks/bench_configs.py fm >> gpurun_out/r5/fm_hot_shards_rate.log 2>&1
  rc=$?; echo "rate hot=$hot rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
