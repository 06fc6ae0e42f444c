#!/bin/bash
# Round 2 call w: 2-rank rehearsal of bench.py's self-launching distributed path on ONE MI355X
# (gloo between the 2 ranks sharing cuda:0; RCCL refuses two ranks per GPU) — both the
# launcher form and the self-launch form the driver's N-GPU run uses.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 HM_DIST_BACKEND=gloo
timeout -k 10 400 python -u bench.py --gpus 2 --steps 12 --warmup 3 > gpurun_out/multirank_selflaunch_r2w.log 2>&1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 12 --warmup 3 > gpurun_out/multirank_torchrun_r2w.log 2>&1
echo done
