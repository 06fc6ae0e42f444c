#!/bin/bash
# Round 2 call o: shared-table linear engine (replicas x waves x reload sweep + tests).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2o}"
timeout -k 10 600 python -u -m pytest tests/test_linear.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_$TAG.log
grep -q "Fatal\|core dumped\|Timeout" gpurun_out/pytest_$TAG.log && exit 3
timeout -k 10 500 python -u benchmarks/linear_shared_probe.py > gpurun_out/linear_shared_$TAG.log 2>&1
echo done
