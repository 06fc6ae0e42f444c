#!/bin/bash
# Round 2 call s: round-health run — full GPU suite, smoke, default bench + kernel stats, SQL
# ingest (Series path), LDA bench.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2s}"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_gpu_$TAG.log
grep -q "Fatal\|core dumped\|Timeout" gpurun_out/pytest_gpu_$TAG.log && exit 3
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_$TAG.log 2>&1
timeout -k 10 600 python -u benchmarks/sql_ingest_bench.py --rows 5000000 > gpurun_out/sql_ingest_$TAG.log 2>&1
timeout -k 10 300 python -u benchmarks/lda_bench.py > gpurun_out/lda_bench_$TAG.log 2>&1
echo done
