#!/bin/bash
# BPR-MF Hogwild concurrency sweep on MI355X: triples/s and sampled AUC per launch grid
# (the default caps the grid at min(users, items) / 256 blocks).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u - > gpurun_out/bpr_grid.log 2>&1 <<'PY'
import json, sys
sys.path.insert(0, "benchmarks")
from bench_configs import bench_bprmf
for g in (0, 212, 424, 848, 1696):
    r = bench_bprmf(opts=f"-grid {g}" if g else "")
    print(json.dumps(r), flush=True)
PY
echo done
