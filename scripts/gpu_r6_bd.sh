#!/bin/bash
# round 6 (second pass, FM past its 1-XCD early ramp: HM_FM_XCDS=6 = the default 6 XCDs, grid 256): counter refresh of the non-FFM hot kernels as shipped now -- BPR's 16-lane float4 form
# (bpr_pf3_kernel<8, 4>), train_fm's fm_pipe_kernel (6 XCDs, grid 256) and GBDT's hist_kernel
set -o pipefail
O=gpurun_out/r6bd
mkdir -p $O
export TMPDIR=/tmp HM_NO_AUTOBUILD=1
G1="FETCH_SIZE"
G2="WRITE_SIZE"
G3="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
G4="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"
G5="TCC_HIT_sum TCC_MISS_sum"
G6="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
run_passes() {   # name, command...
  local name=$1; shift
  local i=0
  for grp in "$G1" "$G2" "$G3" "$G4" "$G5" "$G6"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $O/$name/p$i -o run -- "$@" > $O/${name}_p$i.log 2>&1 || { echo "$name pass $i failed"; tail -5 $O/${name}_p$i.log; return 1; }
    echo "$name pass $i ok"
  done
}
export HM_FM_XCDS=6
run_passes fm python3 benchmarks/pmc_target.py fm || exit 2
python scripts/pmc_summary.py $O/fm fm_pipe 1048576 > $O/fm_summary.json || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace_fm -o run -- python3 benchmarks/pmc_target.py fm > $O/ktrace_fm.log 2>&1 || exit 5
echo ok
