#!/bin/bash
# DP mixing study at the bench's shape on one card (benchmarks/dp_sim.py): N replicas vs one
# replica on the same total rows.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4b
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u benchmarks/dp_sim.py --worlds 2 4 8 --rules mean --lr-power 0 0.5 0.75 1.0 \
  --single-lr 2 2.83 --state fp32 > $O/dp_sim_fp32_lr.jsonl 2>&1
timeout -k 10 600 python -u benchmarks/dp_sim.py --worlds 8 --rules touched precision adasum bmuf --state fp32 \
  > $O/dp_sim_fp32_rules.jsonl 2>&1
