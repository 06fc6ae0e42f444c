#!/bin/bash
# Round 3: FFM grid sweep of the shipped sg12 / sg32 pipelines (default 8,192 blocks = 8 per CU,
# 4 resident): persistent-style 1,024 / 2,048 and 4,096, 16,384, interleaved twice.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
for rep in 1 2; do
  for g in ${GRIDS:-1024 2048 4096 8192 16384}; do
    echo "== grid $g rep $rep" >> gpurun_out/r3ab_grid${TAG:-}.log
    timeout -k 10 200 python -u bench.py --grid $g >> gpurun_out/r3ab_grid${TAG:-}.log 2>&1
  done
done
TAG=${TAG:-} python3 - <<'PY'
import json
lab = None
import os
for l in open("gpurun_out/r3ab_grid" + os.environ.get("TAG", "") + ".log"):
    if l.startswith("=="): lab = l.strip()
    elif l.startswith('{"metric'):
        d = json.loads(l); print(lab, round(d["value"] / 1e6, 1), round(d["value_fp32_state"] / 1e6, 1), d["logloss_heldout"], d["logloss_heldout_fp32"])
PY
