#!/bin/bash
# Same-box A/B: register-resident sg32/sg12 kernels (HM_FFM_VARIANT=6) vs the transposed-image
# pipelines (0), interleaved; a grid sweep of the new kernels; the FFM GPU tests on them.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4c
mkdir -p $O
export HM_NO_AUTOBUILD=1
for rep in 1 2; do
  for v in 0 6; do
    echo "== variant $v rep $rep" >> $O/ab.log
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py --mix-probe 0 >> $O/ab.log 2>&1
  done
done
for g in 4096 16384 32768; do
  echo "== variant 6 grid $g" >> $O/ab.log
  HM_FFM_VARIANT=6 timeout -k 10 300 python -u bench.py --grid $g >> $O/ab.log 2>&1
done
HM_FFM_VARIANT=6 timeout -k 10 600 python -u -m pytest tests/test_ffm.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_ffm_v6.log 2>&1 || true
tail -3 $O/pytest_ffm_v6.log
