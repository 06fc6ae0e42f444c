#!/bin/bash
# train_fm -engine minibatch: GPU test + dense-FM probe
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 300 python -u -m pytest tests/test_fm.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_r2ac.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_r2ac.log
grep -q "Fatal\|core dumped\|Timeout" gpurun_out/pytest_r2ac.log && exit 3
timeout -k 10 600 python -u benchmarks/probes/fm_dense_probe.py > gpurun_out/fm_dense_probe_r2ac.log 2>&1
echo done
