#!/bin/bash
# round 6: counter refresh of the non-FFM hot kernels as shipped now -- BPR's 16-lane float4 form
# (bpr_pf3_kernel<8, 4>), train_fm's fm_pipe_kernel (6 XCDs, grid 256) and GBDT's hist_kernel
set -o pipefail
O=gpurun_out/r6bc
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
run_passes bpr python3 benchmarks/pmc_target.py bprmf || exit 1
python scripts/pmc_summary.py $O/bpr bpr_pf3 20000000 > $O/bpr_summary.json || exit 1
run_passes fm python3 benchmarks/pmc_target.py fm || exit 2
python scripts/pmc_summary.py $O/fm fm_pipe 1048576 > $O/fm_summary.json || exit 2
run_passes gbdt python3 benchmarks/pmc_target.py gbdt || exit 3
python scripts/pmc_summary.py $O/gbdt hist_kernel 2000000 > $O/gbdt_hist_summary.json || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 benchmarks/pmc_target.py bprmf > $O/ktrace_bpr.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace_fm -o run -- python3 benchmarks/pmc_target.py fm > $O/ktrace_fm.log 2>&1 || exit 5
echo ok
