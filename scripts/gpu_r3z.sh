#!/bin/bash
# Round 3: same-box A/B of the fused route + partition count (HM_TREE_FUSE_ROUTE=1) against the
# separate route pass (=0), GBDT and XGBoost configs, interleaved.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
for rep in 1 2; do
  for v in 0 1; do
    echo "== fuse $v rep $rep" >> gpurun_out/r3z_fuse_ab.log
    HM_TREE_FUSE_ROUTE=$v timeout -k 10 300 python -u benchmarks/bench_configs.py gbdt xgboost >> gpurun_out/r3z_fuse_ab.log 2>&1
  done
done
grep -E '^==|ms_per' gpurun_out/r3z_fuse_ab.log | cut -c1-200
echo done
