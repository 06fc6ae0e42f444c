#!/bin/bash
# Generic same-box FFM A/B: FFM GPU tests + smoke, then interleaved bench.py runs of the kernel
# variants in $VARIANTS (HM_FFM_VARIANT), $REPS times.  TAG names the logs.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-ab}"
timeout -k 10 300 python -u -m pytest tests/test_ffm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
for rep in $(seq ${REPS:-2}); do
  for v in ${VARIANTS:-2 0}; do
    echo "== variant $v rep $rep ${BENCH_ARGS:-}" >> gpurun_out/ffm_ab_$TAG.log
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} >> gpurun_out/ffm_ab_$TAG.log 2>&1
  done
done
echo done
