#!/bin/bash
# Counter passes over the fused top-k kernel (benchmarks/mips_prof_target.py).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-x}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_WAVES SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_FLAT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/mips_pmc_$TAG/p$i -o run -- python3 benchmarks/mips_prof_target.py > gpurun_out/mips_pmc_${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/mips_pmc_${TAG}_p$i.log; exit 1; }
done
python scripts/pmc_summary.py gpurun_out/mips_pmc_$TAG mips_topk 1 > gpurun_out/mips_pmc_$TAG.json
echo done
