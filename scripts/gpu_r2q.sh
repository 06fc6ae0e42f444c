#!/bin/bash
# Round 2 call q: fused join-predict on the GPU (test + bench), bench-scale parity on the CPU
# generator's stream (bf16 + fp32 state).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2q}"
timeout -k 10 300 python -u -m pytest tests/test_sql_fused.py tests/test_sql.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_$TAG.log
grep -q "Fatal\|core dumped\|Timeout" gpurun_out/pytest_$TAG.log && exit 3
timeout -k 10 400 python -u benchmarks/sql_predict_bench.py --rows 1000000 --generic-rows 50000 --device cuda > gpurun_out/sql_predict_$TAG.log 2>&1
timeout -k 10 400 python -u bench.py --gen-device cpu > gpurun_out/bench_cpugen_bf16_$TAG.log 2>&1
timeout -k 10 400 python -u bench.py --gen-device cpu --state fp32 > gpurun_out/bench_cpugen_fp32_$TAG.log 2>&1
echo done
