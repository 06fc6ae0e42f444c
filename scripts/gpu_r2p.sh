#!/bin/bash
# Round 2 call p: linear shared-engine tests + config, FFM bench bf16/fp32 (parity record),
# rocprof kernel trace of the SQL ingest path.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2p}"
timeout -k 10 600 python -u -m pytest tests/test_linear.py tests/test_ingest.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_$TAG.log
grep -q "Fatal\|core dumped\|Timeout" gpurun_out/pytest_$TAG.log && exit 3
timeout -k 10 300 python -u benchmarks/bench_configs.py linear_hashed > gpurun_out/configs_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_bf16_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --state fp32 > gpurun_out/bench_fp32_$TAG.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ingest_$TAG -o run -- \
  python3 benchmarks/sql_ingest_bench.py --rows 1000000 > gpurun_out/prof_ingest_$TAG.log 2>&1
echo done
