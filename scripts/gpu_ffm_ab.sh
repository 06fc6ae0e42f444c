#!/bin/bash
# Same-box A/B of the FFM kernel: hivemall_amd/_lib_ab/libhm_hip_base.so (baseline) against the
# in-tree library, interleaved bench.py runs, then the FFM GPU tests on the new library.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-x}"
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export HM_HIP_LIB=$PWD/hivemall_amd/_lib_ab/libhm_hip_base.so; else unset HM_HIP_LIB; fi
    echo "== $v rep $rep" >> gpurun_out/ffm_ab_$TAG.log
    timeout -k 10 300 python -u bench.py >> gpurun_out/ffm_ab_$TAG.log 2>&1
  done
done
unset HM_HIP_LIB
timeout -k 10 600 python -u -m pytest tests/test_ffm.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_ffm_$TAG.log 2>&1
echo done
