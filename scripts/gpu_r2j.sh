#!/bin/bash
# Round 2 call j: FFM A/B (DPP sums, branch-free slot decode) + GPU tests of the new pieces
# (many-class trees, mix kernels, MF) + smoke.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2j}"
timeout -k 10 600 python -u -m pytest tests/test_trees.py tests/test_mf.py tests/test_mix_lowp.py tests/test_ffm.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
for rep in 1 2; do
  for v in 2 0; do
    echo "== variant $v rep $rep" >> gpurun_out/ffm_ab_$TAG.log
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py >> gpurun_out/ffm_ab_$TAG.log 2>&1
  done
done
echo done
