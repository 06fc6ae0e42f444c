#!/bin/bash
# FFM fp32 sg32: next row's G in registers (variant 10: 53 KB LDS, 3 blocks per CU) vs the LDS
# landing zone (default), interleaved; GPU FFM tests under variant 10; linear RELOAD A/B at 8
# rows in flight; tree tests (leaf sums with per-wave copies) and GBDT.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5a
mkdir -p $O
export HM_NO_AUTOBUILD=1
HM_FFM_VARIANT=10 timeout -k 10 600 python -u -m pytest tests/test_ffm.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/pytest_ffm_v10.log 2>&1
tail -1 $O/pytest_ffm_v10.log
for rep in 1 2; do
  for v in 0 10; do
    echo "== ffm variant $v rep $rep" >> $O/ffm_ab.log
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py --mix-probe 0 --alt-run 0 >> $O/ffm_ab.log 2>&1
  done
done
echo "== ffm variant 10 same stream" >> $O/ffm_ab.log
HM_FFM_VARIANT=10 timeout -k 10 300 python -u bench.py --gen-device cpu --mix-probe 0 --alt-run 0 >> $O/ffm_ab.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_trees.py \
  tests/test_xgboost.py > $O/pytest_trees.log 2>&1
timeout -k 10 300 python -u benchmarks/bench_configs.py gbdt > $O/gbdt.log 2>&1
for r in 1 0; do
  HM_LINEAR_RELOAD=$r timeout -k 10 600 python -u benchmarks/linear_rules_parity.py 1000000 "-opt adam -eta0 0.01" \
    "-opt sgd -eta0 0.05" > $O/linear_reload$r.jsonl 2>&1
done
