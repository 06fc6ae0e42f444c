#!/bin/bash
# FFM: sg32 without pad stores is the default now; bf16 sg12 without pad stores (variant 8) A/B.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5p
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ffm.py > $O/pytest_ffm.log 2>&1
for rep in 1 2 3; do
  for v in 0 8; do
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py --state bf16 --alt-run 0 --steps 40 --warmup 5 > $O/bench_bf16_v${v}_r${rep}.log 2>&1
    echo "bf16 variant $v rep $rep: $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*' $O/bench_bf16_v${v}_r${rep}.log | tr '\n' ' ')" >> $O/ab.log
  done
done
timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1
tail -1 $O/bench_default.log | cut -c1-200
