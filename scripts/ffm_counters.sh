#!/bin/bash
# rocprofv3 hardware-counter passes over the FFM kernel (one counter group per run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HM_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT="${OUT:-ffm_pmc_packed}"
PAT="${PAT:-ffm_packed}"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/$OUT/p$i -o run -- python3 benchmarks/ffm_prof_target.py > gpurun_out/${OUT}_p$i.log 2>&1 || { echo "pass $i failed: $?"; tail -5 gpurun_out/${OUT}_p$i.log; exit 1; }
done
python scripts/pmc_summary.py gpurun_out/$OUT $PAT > gpurun_out/${OUT}_summary.json
cat gpurun_out/${OUT}_summary.json
