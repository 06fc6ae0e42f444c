# round 5 validation: the full GPU suite, smoke, and the default bench
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r5/pytest_gpu_val.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5/pytest_gpu_val.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5/smoke_val.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r5/smoke_val.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r5/bench_val.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/r5/bench_val.log | cut -c1-300
