#!/bin/bash
# round 6: the bf16 kernel's phase-B landing-zone read kept as one ds_read_b128 (the compiler had
# narrowed it to a 2-way b64 + 4-way b32 pair): LDS counters (plain and side-table linear steps)
# and three bench runs
set -o pipefail
O=gpurun_out/r6az
mkdir -p $O
export TMPDIR=/tmp HM_NO_AUTOBUILD=1
for la in 0 4; do
  HM_FFM_LIN_ATOMIC=$la BF16=1 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_la$la -o run -- python3 benchmarks/ffm_prof_target.py > $O/pmc_la$la.log 2>&1 || exit 1
  python scripts/pmc_summary.py $O/pmc_la$la sg12 > $O/pmc_la$la.json || exit 1
  python -c "import json; d=json.load(open('$O/pmc_la$la.json')); print('lin_atomic=$la', d['kernel'].get('kernel','')[40:95], d['mean_per_dispatch'])"
done
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench$i.json 2> $O/bench$i.err || exit 2
  python -c "import json; d=json.load(open('$O/bench$i.json')); print('bench', d['value'], d['logloss_gap'], d['value_bf16_state'], d['logloss_gap_bf16'])"
done
echo ok
