#!/bin/bash
# round 6: bf16 kernel slot DMA as 16 B (dwordx4, over-reading the next slot's first dword) instead
# of 12 B (dwordx3): same 16-B landing stride; LDS conflict counters + interleaved bench A/B
set -o pipefail
O=gpurun_out/r6ai
mkdir -p $O
export TMPDIR=/tmp HM_NO_AUTOBUILD=1
for v in 0 11; do
  BF16=1 HM_FFM_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_v$v -o run -- python3 benchmarks/ffm_prof_target.py > $O/pmc_v$v.log 2>&1 || exit 1
  python scripts/pmc_summary.py $O/pmc_v$v sg12 > $O/pmc_v${v}_summary.json || exit 1
  python -c "import json; d=json.load(open('$O/pmc_v${v}_summary.json'))['mean_per_dispatch']; print('v$v', d)"
done
for rep in 1 2 3; do for v in 0 11; do
  HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --state bf16 --alt-run 0 > $O/bench_v${v}_$rep.log 2>&1 || exit 2
  tail -1 $O/bench_v${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('v$v', d['value'], d.get('logloss_gap'))"
done; done
echo ok
