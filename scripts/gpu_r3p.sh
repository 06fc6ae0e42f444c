#!/bin/bash
# Round 3: SQL feature engineering + train_classifier end to end on the GPU (1M Criteo-shaped string rows).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 400 python -u benchmarks/sql_ftvec_bench.py 1000000 cuda arrow 2>&1 | tee gpurun_out/r3p_sql_ftvec_gpu.log
