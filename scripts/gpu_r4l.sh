#!/bin/bash
# Round 4: kernel-time stats + counter passes of the non-FFM hot kernels after the round-4 changes
# (hist_kernel / hist_sibling / level_finalize, fm_pipe_kernel, bpr_kernel, mf_kernel).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
export TMPDIR=/tmp
for tgt in ${TARGETS:-gbdt fm bprmf mf}; do
  OUT=gpurun_out/pmc_r4_$tgt
  mkdir -p $OUT
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 benchmarks/pmc_target.py $tgt > $OUT/stats.log 2>&1
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 benchmarks/pmc_target.py $tgt > $OUT/p$i.log 2>&1
  done
  echo "$tgt done"
done
