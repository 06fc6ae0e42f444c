#!/bin/bash
# Multi-rank rehearsal of bench.py's distributed path on ONE MI355X: 2 ranks share cuda:0 and
# mix over gloo (RCCL refuses two ranks per GPU).  Checks the OverlappedMixer / barrier / max-
# over-ranks code with real device tensors; the throughput number is meaningless.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 HM_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 12 --warmup 3 > gpurun_out/multirank_rehearsal.log 2>&1
echo done
