#!/bin/bash
# Round 3: SQL / linear GPU tests after the Arrow-backed model-table names, then the SQL
# feature-engineering + train_classifier statement on 1 M rows end to end.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 500 python -u -m pytest tests/test_sql.py tests/test_sql_fused.py tests/test_sql_dist.py tests/test_linear.py tests/test_ingest.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3aa_pytest_sql.log 2>&1
tail -2 gpurun_out/r3aa_pytest_sql.log
timeout -k 10 400 python -u benchmarks/sql_ftvec_bench.py 1000000 cuda arrow 2>&1 | tee gpurun_out/r3aa_sql_ftvec_gpu.log
