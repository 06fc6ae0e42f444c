#!/bin/bash
# Round 2 call k: device-side ingest (tests, SQL train_ffm over 5M string rows, rocprof of the
# ingest kernels), FFM -w0 atomic bias test, smoke, default bench.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2k}"
timeout -k 10 600 python -u -m pytest tests/test_ingest.py tests/test_ffm.py tests/test_fm.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 600 python -u benchmarks/sql_ingest_bench.py --rows 5000000 --host-rows 200000 > gpurun_out/sql_ingest_$TAG.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ingest_$TAG -o run -- \
  python3 benchmarks/sql_ingest_bench.py --rows 1000000 > gpurun_out/prof_ingest_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
echo done
