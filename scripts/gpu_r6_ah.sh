#!/bin/bash
# round 6: counters of the side-table (default) fp32 / bf16 FFM kernels beside the plain-store
# kernels (HM_FFM_LIN_ATOMIC=0), at the driver's config
set -o pipefail
O=gpurun_out/r6ah
mkdir -p $O
export TMPDIR=/tmp HM_NO_AUTOBUILD=1
G1="FETCH_SIZE"
G2="WRITE_SIZE"
G3="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
G4="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"
G5="TCC_HIT_sum TCC_MISS_sum"
G6="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
run_passes() {   # name, env, command...
  local name=$1; shift; local envs=$1; shift
  local i=0
  for grp in "$G1" "$G2" "$G3" "$G4" "$G5" "$G6"; do
    i=$((i+1))
    env $envs timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/$name/p$i -o run -- "$@" > $O/${name}_p$i.log 2>&1 || { echo "$name pass $i failed"; return 1; }
  done
}
run_passes sg32_side "BF16=0" python3 benchmarks/ffm_prof_target.py || exit 1
run_passes sg32_plain "BF16=0 HM_FFM_LIN_ATOMIC=0" python3 benchmarks/ffm_prof_target.py || exit 2
run_passes sg12_side "BF16=1" python3 benchmarks/ffm_prof_target.py || exit 3
python scripts/pmc_summary.py $O/sg32_side sg32 > $O/sg32_side_summary.json || exit 4
python scripts/pmc_summary.py $O/sg32_plain sg32 > $O/sg32_plain_summary.json || exit 4
python scripts/pmc_summary.py $O/sg12_side sg12 > $O/sg12_side_summary.json || exit 4
echo ok
