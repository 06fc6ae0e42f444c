#!/bin/bash
# FFM tests incl. the polled-variant grid-1 test, smoke, dense-FM probe
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_r2aa.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_r2aa.log
grep -q "Fatal\|core dumped\|Timeout\|rc=" gpurun_out/pytest_r2aa.log && exit 3
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r2aa.log 2>&1
timeout -k 10 400 python -u benchmarks/probes/fm_dense_probe.py > gpurun_out/fm_dense_probe.log 2>&1
echo done
