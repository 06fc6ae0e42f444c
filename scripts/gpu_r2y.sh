#!/bin/bash
# Round 2 call y: FFM sink variant with same-lane FTRL forwarding (tests, smoke, A/B vs
# variant 3), then the dense-FM probe (per-row kernel vs mini-batch MFMA GEMMs).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2y}"
timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_$TAG.log
grep -q "Fatal\|core dumped\|Timeout\|rc=" gpurun_out/pytest_$TAG.log && exit 3
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
for rep in 1 2 3; do
  for v in 0 3; do
    echo "== variant $v rep $rep" >> gpurun_out/ffm_ab_$TAG.log
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py >> gpurun_out/ffm_ab_$TAG.log 2>&1
  done
done
timeout -k 10 400 python -u benchmarks/probes/fm_dense_probe.py > gpurun_out/fm_dense_probe_$TAG.log 2>&1
echo done
