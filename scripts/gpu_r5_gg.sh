# round 5 gg: sharded global-bias FTRL state (-w0) -- FFM tests, rate with / without -w0
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/r5/pytest_ffm_gg.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/r5/pytest_ffm_gg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u benchmarks/ffm_w0_rate_probe.py > gpurun_out/r5/ffm_w0_rate_sharded.jsonl 2> gpurun_out/r5/ffm_w0_rate_sharded.err
echo "probe rc=$?"
