#!/bin/bash
# FFM fp32 kernel with the block's own updates forwarded into its prefetched next row: tests,
# rate, same-stream parity (sequential 0.44501), early-training parity at 500 K rows; trees with
# deferred materialisation.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4x
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests/test_ffm.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_ffm.log 2>&1
tail -3 $O/pytest_ffm.log
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --mix-probe 0 >> $O/bench.log 2>&1
done
timeout -k 10 300 python -u bench.py --gen-device cpu --mix-probe 0 > $O/bench_same_stream.log 2>&1
timeout -k 10 900 python -u benchmarks/ffm_early_parity.py 500000 0 > $O/ffm_early.jsonl 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_trees.py \
  tests/test_xgboost.py > $O/pytest_trees.log 2>&1
timeout -k 10 300 python -u benchmarks/bench_configs.py gbdt xgboost > $O/gbdt.log 2>&1
