#!/bin/bash
# A/Bs of round-4 kernel variants, same box, interleaved:
#  trees: histogram kernel in isolation (packed 64-bit LDS adds vs 32-bit), GBDT with the fused
#   route + partition count (default) and packed histograms, tree tests under the packed kernel;
#  FFM fp32 512-thread blocks (HM_FFM_VARIANT=8) vs 256 (0), rate + same-stream parity;
#  FM coherent loads/stores (HM_FM_COH=1) at the default grid and at 512 blocks;
#  linear shared engine coherent stores (HM_LINEAR_COH=1) on three rules.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4h
mkdir -p $O
export HM_NO_AUTOBUILD=1
for pk in 0 1; do
  HM_HIST_PACK=$pk timeout -k 10 300 python -u benchmarks/hist_micro.py >> $O/hist_micro.jsonl 2>> $O/hist_micro.err
done
for cfg in "0 0 0" "1 0 0" "1 1 0" "1 1 1" "1 0 1"; do
  set -- $cfg
  echo "== route_fused $1 hist_pack $2 hist_wide $3" >> $O/gbdt_ab.log
  HM_ROUTE_FUSED=$1 HM_HIST_PACK=$2 HM_HIST_WIDE=$3 timeout -k 10 300 python -u benchmarks/bench_configs.py gbdt xgboost >> $O/gbdt_ab.log 2>&1
done
HM_HIST_PACK=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_trees.py tests/test_xgboost.py > $O/pytest_trees_pack.log 2>&1
for rep in 1 2; do
  for v in 0 8; do
    echo "== ffm variant $v rep $rep" >> $O/ffm_ab.log
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py --mix-probe 0 --alt-run 0 >> $O/ffm_ab.log 2>&1
  done
done
for g in 4096 16384 32768; do
  echo "== ffm variant 0 grid $g" >> $O/ffm_ab.log
  timeout -k 10 300 python -u bench.py --mix-probe 0 --alt-run 0 --grid $g >> $O/ffm_ab.log 2>&1
done
echo "== ffm variant 8 same stream" >> $O/ffm_ab.log
HM_FFM_VARIANT=8 timeout -k 10 300 python -u bench.py --gen-device cpu --mix-probe 0 --alt-run 0 >> $O/ffm_ab.log 2>&1
for c in 0 1; do
  for g in "" "-grid 512"; do
    echo "== fm coh $c opts $g" >> $O/fm_coh.log
    HM_FM_COH=$c HM_BENCH_FM_OPTS="$g" timeout -k 10 300 python -u benchmarks/bench_configs.py fm >> $O/fm_coh.log 2>&1
  done
done
for c in 0 1; do
  HM_LINEAR_COH=$c timeout -k 10 600 python -u benchmarks/linear_rules_parity.py 1000000 "-opt adagrad" "-opt adam" \
    "-opt momentum -eta0 0.05" > $O/linear_coh$c.jsonl 2>&1
done
HM_FFM_VARIANT=8 timeout -k 10 600 python -u -m pytest tests/test_ffm.py -m gpu -v --timeout 300 --timeout-method thread \
  > $O/pytest_ffm_v8.log 2>&1 || true
tail -3 $O/pytest_ffm_v8.log
