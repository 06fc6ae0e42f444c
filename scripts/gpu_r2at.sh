#!/bin/bash
# Tree builder: node arrays written in place by the level kernel (no per-level concatenations),
# importance in-kernel, RF OOB read once per fit; tree GPU tests, GBDT/RF configs, RF trace
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 400 python -u -m pytest tests/test_trees.py tests/test_xgboost.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_trees_r2at.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_trees_r2at.log
grep -q "Fatal\|core dumped\|Timeout\|rc=" gpurun_out/pytest_trees_r2at.log && exit 3
timeout -k 10 200 python -u benchmarks/probes/rf_prof_target.py 10 > gpurun_out/rf_wall_r2at.log 2>&1
timeout -k 10 200 python -u benchmarks/probes/gbt_prof_target.py 20 > gpurun_out/gbt_wall_r2at.log 2>&1
timeout -k 10 400 python -u benchmarks/bench_configs.py gbdt rf > gpurun_out/configs_trees_r2at.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rf2 -o run -- \
  python3 benchmarks/probes/rf_prof_target.py 10 > gpurun_out/prof_rf2.log 2>&1
echo done
