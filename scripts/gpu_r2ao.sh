#!/bin/bash
# GBT fused level finalisation: tree GPU tests, GBDT/RF configs, kernel breakdown
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 400 python -u -m pytest tests/test_trees.py tests/test_xgboost.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_trees_r2ao.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_trees_r2ao.log
grep -q "Fatal\|core dumped\|Timeout" gpurun_out/pytest_trees_r2ao.log && exit 3
timeout -k 10 400 python -u benchmarks/bench_configs.py gbdt rf > gpurun_out/configs_trees_r2ao.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gbt3 -o run -- \
  python3 benchmarks/probes/gbt_prof_target.py 20 > gpurun_out/prof_gbt3.log 2>&1
echo done
