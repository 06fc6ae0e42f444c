#!/bin/bash
# Round 3: 2-rank rehearsal of the BASELINE configs 4 and 5 harness (bench_configs.py --gpus 2)
# on ONE MI355X: gloo between the ranks sharing cuda:0 (RCCL refuses two ranks per card), full
# shapes; row-sharded GBDT / XGBoost with per-level histogram all-reduce, per-rank RF trees,
# BPR with replica mixing.  Times are meaningless (both ranks share one GPU and gloo moves the
# collectives through host memory); the output shows the multi-rank GPU path runs end to end.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 HM_DIST_BACKEND=gloo
( while sleep 30; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u benchmarks/bench_configs.py --gpus 2 gbdt xgboost rf bprmf > gpurun_out/configs_dist_w2_r3w.log 2>&1
grep '^{' gpurun_out/configs_dist_w2_r3w.log | cut -c1-300
echo done
