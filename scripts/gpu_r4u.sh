#!/bin/bash
# FFM fp32 paired-slot kernel (HM_FFM_VARIANT=9) vs the default: rate, held-out logloss, the
# GPU FFM tests under it; the linear 2^24 parity test after AdaDelta's routing.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4u
mkdir -p $O
export HM_NO_AUTOBUILD=1
HM_FFM_VARIANT=9 timeout -k 10 600 python -u -m pytest tests/test_ffm.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_ffm_v9.log 2>&1
tail -3 $O/pytest_ffm_v9.log
for rep in 1 2; do
  for v in 0 9; do
    echo "== ffm variant $v rep $rep" >> $O/ffm_ab.log
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py --mix-probe 0 --alt-run 0 >> $O/ffm_ab.log 2>&1
  done
done
echo "== ffm variant 9 same stream" >> $O/ffm_ab.log
HM_FFM_VARIANT=9 timeout -k 10 300 python -u bench.py --gen-device cpu --mix-probe 0 --alt-run 0 >> $O/ffm_ab.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
HM_FFM_VARIANT=9 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_v9 -o ffm -- \
  python3 bench.py --mix-probe 0 --alt-run 0 > $O/prof_v9.log 2>&1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_linear.py \
  -k "hashed_2p24" > $O/pytest_2p24.log 2>&1 || true
grep -E "FAILED|passed|failed" $O/pytest_2p24.log | tail -3
