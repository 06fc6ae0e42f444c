#!/bin/bash
# FFM: polled early-gather kernel (variant 5) at reduced grids vs the default, same box
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
for rep in 1 2; do
  for cfg in "3 0" "5 0" "5 768" "5 512" "3 768"; do
    set -- $cfg
    echo "== variant $1 grid $2 rep $rep" >> gpurun_out/ffm_grid_ab_r2ad.log
    HM_FFM_VARIANT=$1 timeout -k 10 300 python -u bench.py --grid $2 >> gpurun_out/ffm_grid_ab_r2ad.log 2>&1
  done
done
echo done
