#!/bin/bash
# rocprofv3 counter passes (one group per run) + kernel stats of the fp32 headline kernel
# (ffm_pipe_sg32_kernel) at the driver's config (criteo_ffm rows: fld / val DMAs); MODES lists
# kernel variants (0 = default); summaries into gpurun_out/r5/pmc_sg32_v<variant>_summary.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HM_NO_AUTOBUILD=1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
for v in ${MODES:-0}; do
  export HM_FFM_VARIANT=$v
  OUT=r5/pmc_sg32_v$v
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$OUT/ks -o run -- python3 benchmarks/ffm_prof_target.py > gpurun_out/${OUT}_ks.log 2>&1 || { echo "stats v$v failed: $?"; exit 1; }
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/$OUT/p$i -o run -- python3 benchmarks/ffm_prof_target.py > gpurun_out/${OUT}_p$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "pass v$v $i failed: $rc"; tail -3 gpurun_out/${OUT}_p$i.log; exit 1; fi
  done
  python scripts/pmc_summary.py gpurun_out/$OUT ffm_pipe_sg32 > gpurun_out/${OUT}_summary.json
  cat gpurun_out/${OUT}_summary.json
done
