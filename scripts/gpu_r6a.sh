#!/bin/bash
# Trees: blocks of the fused route + count pass (HM_ROUTE_GRID) A/B on GBDT / XGBoost.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6a
mkdir -p $O
export HM_NO_AUTOBUILD=1
for rep in 1 2; do
  for g in 1024 512 2048; do
    echo "== HM_ROUTE_GRID=$g rep $rep" >> $O/trees_ab.log
    HM_ROUTE_GRID=$g timeout -k 10 300 python -u benchmarks/bench_configs.py gbdt xgboost >> $O/trees_ab.log 2>&1
  done
done
