# round 5 ae: -w0 after skipping the first-row shard re-read, every 32: rates (bf16 at several grids), single-block -w0 test
set -o pipefail
mkdir -p gpurun_out/r5
export HM_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_ffm.py -m gpu -x -v --timeout 200 --timeout-method thread -k "single_block or global_bias" > gpurun_out/r5/pytest_ffm_ae.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/r5/pytest_ffm_ae.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/ffm_option_rate_sweep.py "-c" "-c -w0" "-c -bf16_state" "-c -bf16_state -w0" "-c -bf16_state -w0 -grid 4096" "-c -bf16_state -w0 -grid 1024" "-c -bf16_state -grid 1024" > gpurun_out/r5/ffm_w0_ae.jsonl 2>/dev/null
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/r5/ffm_w0_ae.jsonl
