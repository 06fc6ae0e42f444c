#!/bin/bash
# Health run after the MF/FFM changes: all GPU tests, smoke, bench, MF probe at the new default grid
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r2al.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_gpu_r2al.log
grep -q "Fatal\|core dumped\|Timeout" gpurun_out/pytest_gpu_r2al.log && exit 3
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r2al.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r2al.log 2>&1
timeout -k 10 400 python -u benchmarks/mf_atomic_probe.py ml20m > gpurun_out/mf_atomic_probe_r2al.log 2>&1
echo done
