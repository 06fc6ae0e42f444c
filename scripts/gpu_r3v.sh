#!/bin/bash
# Round 3: 8-rank rehearsal of bench.py's GPU path on ONE MI355X (gloo; the 8 ranks share cuda:0,
# so rows/s are meaningless): held-out logloss of the mixed model at N = 8.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 HM_DIST_BACKEND=gloo
( while sleep 30; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 8 --steps 20 --warmup 5 --fp32-run 0 --mix-probe 1 > gpurun_out/multirank_torchrun_w8_r3v.log 2>&1
grep '^{"metric' gpurun_out/multirank_torchrun_w8_r3v.log | cut -c1-300
echo done
