#!/bin/bash
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests/test_trees.py tests/test_xgboost.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_e.log 2>&1
timeout -k 10 600 python -u benchmarks/bench_configs.py gbdt rf > gpurun_out/configs_e.log 2>&1
timeout -k 10 600 python -u benchmarks/bench_configs.py gbdt --profile > gpurun_out/configs_e_prof.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_e.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_e -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_e.log 2>&1
echo done
