#!/bin/bash
# round 6: sg32 KEEP variant (slot metadata in registers) exactness + interleaved bench A/B + LDS
# counters; BPR three-stage pipeline A/B + tests; FM hot write-through on 1 of N updates
set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python benchmarks/ffm_variant_exact.py 0 9 > $O/keep_exact.jsonl 2> $O/keep_exact.err || exit 1
for rep in 1 2 3; do
  for v in 0 9; do
    HM_FFM_VARIANT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --alt-run 0 > $O/bench_v${v}_r$rep.log 2>&1 || exit 2
  done
done
for v in 0 9; do
  HM_FFM_VARIANT=$v timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_lds_v$v -o run -- python3 benchmarks/ffm_prof_target.py > $O/pmc_lds_v$v.log 2>&1 || exit 3
done
for v in 2 0 2 0; do
  HM_BPR_VARIANT=$v timeout -k 10 300 python benchmarks/bench_configs.py bprmf > $O/bpr_v$v.log 2>&1 || exit 4
  cat $O/bpr_v$v.log >> $O/bpr_ab.log
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_mf.py -k "bpr" > $O/pytest_bpr.log 2>&1 || exit 5
for ev in 16 64; do
  HM_FM_HOT_FRAC=0.002 HM_FM_HOT_EVERY=$ev HM_BENCH_FM_OPTS="-grid 256" timeout -k 10 200 python benchmarks/bench_configs.py fm > $O/fm_rate_e${ev}_g256.log 2>&1 || exit 6
done
PROBE_HOT=0.002 PROBE_HOT_EVERY=16,64 PROBE_REPS=1 timeout -k 10 300 python -u benchmarks/fm_grid_parity_probe.py 256 > $O/fm_hot_every_parity.jsonl 2> $O/fm_hot_every_parity.err || exit 7
echo ok
