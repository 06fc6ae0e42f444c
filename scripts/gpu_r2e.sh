#!/bin/bash
# Round 2 call e: FFM memory roofline probe + pipe kernel (slot meta once per row) A/B.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2e}"
timeout -k 10 300 python -u benchmarks/ffm_mem_roofline.py > gpurun_out/ffm_roofline_$TAG.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_ffm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
for rep in 1 2; do
  for v in 2 0; do
    echo "== variant $v state bf16 rep $rep" >> gpurun_out/ffm_ab_$TAG.log
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py >> gpurun_out/ffm_ab_$TAG.log 2>&1
  done
done
echo done
