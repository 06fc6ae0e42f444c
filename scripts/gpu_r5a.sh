#!/bin/bash
# FFM fp32 sg32 with the next row's G in registers (53 KB LDS: 3 blocks per CU): tests, rate,
# same-stream parity, kernel stats.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5a
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests/test_ffm.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_ffm.log 2>&1
tail -3 $O/pytest_ffm.log
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py --mix-probe 0 >> $O/bench.log 2>&1
done
timeout -k 10 300 python -u bench.py --gen-device cpu --mix-probe 0 --alt-run 0 > $O/bench_same_stream.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o ffm -- \
  python3 bench.py --mix-probe 0 --alt-run 0 > $O/prof.log 2>&1
