#!/bin/bash
# round 6: BPR (config 5) grid with the 16-lane float4 kernel -- the 852-block default (1 block per
# 32 items) dates from the one-triple-per-wave kernel; rate and sampled AUC at 852 .. 3,408 blocks
set -o pipefail
O=gpurun_out/r6be
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python - > $O/bpr_grid.jsonl 2> $O/bpr_grid.err <<'PY' || { tail -5 $O/bpr_grid.err; exit 1; }
import json, sys
sys.path.insert(0, ".")
from benchmarks import bench_configs as bc
for rep in range(2):
    for g in (852, 1278, 1704, 2556, 3408):
        r = bc.bench_bprmf(opts=f"-grid {g}")
        print(json.dumps({"grid": g, "rep": rep, "triples_per_s": r["triples_per_s"], "auc": r["sampled_auc"]}), flush=True)
PY
cat $O/bpr_grid.jsonl
echo ok
