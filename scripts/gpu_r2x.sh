#!/bin/bash
# Round 2 call x: FFM pipe kernel with the store sink (vmcnt(NS) instead of vmcnt(0) at the row
# top) — FFM GPU tests + smoke, then same-box interleaved A/B vs variant 3 (no sink).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2x}"
timeout -k 10 400 python -u -m pytest tests/test_ffm.py tests/test_ingest.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_$TAG.log
grep -q "Fatal\|core dumped\|Timeout\|rc=" gpurun_out/pytest_$TAG.log && exit 3
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
for rep in 1 2 3; do
  for v in 0 3; do
    echo "== variant $v rep $rep" >> gpurun_out/ffm_ab_$TAG.log
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py >> gpurun_out/ffm_ab_$TAG.log 2>&1
  done
done
echo done
