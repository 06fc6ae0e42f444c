#!/bin/bash
# Round 2 call m: device parser probe, ingest + linear shared-engine + FFM -w0 tests, hashed
# linear config, SQL ingest bench, smoke, default bench.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2m}"
timeout -k 10 120 python -u benchmarks/parse_probe.py > gpurun_out/parse_probe_$TAG.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_ingest.py tests/test_linear.py tests/test_ffm.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_$TAG.log
grep -q "Fatal\|core dumped\|Timeout" gpurun_out/pytest_$TAG.log && exit 3
timeout -k 10 300 python -u benchmarks/bench_configs.py linear_hashed > gpurun_out/configs_$TAG.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 600 python -u benchmarks/sql_ingest_bench.py --rows 5000000 --host-rows 200000 > gpurun_out/sql_ingest_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
echo done
