#!/bin/bash
# Hardware counters of the FM dense gradient kernels (MFMA vs VALU), one counter group per pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=fmd_pmc
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/$OUT/p$i -o run -- python3 benchmarks/probes/fmd_prof_target.py > gpurun_out/${OUT}_p$i.log 2>&1 || { echo "pass $i failed: $?"; tail -5 gpurun_out/${OUT}_p$i.log; exit 1; }
done
python scripts/pmc_summary.py gpurun_out/$OUT fmd_mfma 65536 > gpurun_out/${OUT}_mfma_summary.json
python scripts/pmc_summary.py gpurun_out/$OUT fmd_grad 65536 > gpurun_out/${OUT}_valu_summary.json
cat gpurun_out/${OUT}_mfma_summary.json gpurun_out/${OUT}_valu_summary.json
