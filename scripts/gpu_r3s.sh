#!/bin/bash
# Round 3: histogram statistic pairs as one ds_add_u64 (trees.hip hist_kernel): tree/xgboost GPU
# tests, then gbdt / xgboost / rf bench configs, baseline library vs new, interleaved.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_trees.py tests/test_xgboost.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3s_pytest_trees.log 2>&1
tail -2 gpurun_out/r3s_pytest_trees.log
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export HM_HIP_LIB=$PWD/hivemall_amd/_lib_ab/libhm_hip_base.so; else unset HM_HIP_LIB; fi
    echo "== $v rep $rep" >> gpurun_out/r3s_trees_ab.log
    timeout -k 10 300 python -u benchmarks/bench_configs.py gbdt xgboost >> gpurun_out/r3s_trees_ab.log 2>&1
  done
done
unset HM_HIP_LIB
timeout -k 10 300 python -u benchmarks/bench_configs.py rf >> gpurun_out/r3s_trees_ab.log 2>&1
echo done
