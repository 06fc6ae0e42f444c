#!/bin/bash
# round 6: where the bf16 kernel's LDS bank conflicts come from — LDS counters of the sg12 kernel
# at KEEP 0 / 1 / 2 (plain linear stores), beside sg32
set -o pipefail
O=gpurun_out/r6at
mkdir -p $O
export TMPDIR=/tmp HM_NO_AUTOBUILD=1
export HM_FFM_LIN_ATOMIC=0
for cfg in "1 9" "1 10" "1 0" "0 0"; do
  set -- $cfg
  BF16=$1 HM_FFM_VARIANT=$2 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_b$1_v$2 -o run -- python3 benchmarks/ffm_prof_target.py > $O/pmc_b$1_v$2.log 2>&1 || exit 1
  pat=sg12; [ $1 = 0 ] && pat=sg32
  python scripts/pmc_summary.py $O/pmc_b$1_v$2 $pat > $O/pmc_b$1_v$2.json || exit 1
  python -c "import json; d=json.load(open('$O/pmc_b$1_v$2.json')); m=d['mean_per_dispatch']; print('bf16=$1 v$2', d['kernel'].get('kernel','')[40:95], m)"
done
(unset HM_FFM_LIN_ATOMIC; timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err) || exit 1
cat $O/bench.json
echo ok
