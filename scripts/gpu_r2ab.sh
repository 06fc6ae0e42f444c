#!/bin/bash
# Full GPU test suite + smoke + default bench (round-end health check)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu_r2ab.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_gpu_r2ab.log
grep -q "Fatal\|core dumped\|Timeout" gpurun_out/pytest_gpu_r2ab.log && exit 3
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r2ab.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r2ab.log 2>&1
echo done
