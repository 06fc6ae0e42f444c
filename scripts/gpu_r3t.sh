#!/bin/bash
# Round 3: multi-rank rehearsal of bench.py on ONE MI355X (gloo between ranks sharing cuda:0;
# RCCL refuses two ranks per GPU): the self-launch form the driver's N-GPU run uses at N = 2
# and the torchrun form at N = 4.  Exercises the GPU side of the overlapped shard-mean mix
# (pack3 / merge3 kernels, side stream, fused repack) across ranks.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 HM_DIST_BACKEND=gloo
# heartbeat: gloo moves the 340-MB mixes through host memory, so a run can be quiet for minutes
( while sleep 30; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/multirank_selflaunch_w2_r3t.log 2>&1
tail -1 gpurun_out/multirank_selflaunch_w2_r3t.log | cut -c1-300
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 4 --steps 20 --warmup 5 --fp32-run 0 > gpurun_out/multirank_torchrun_w4_r3t.log 2>&1
tail -1 gpurun_out/multirank_torchrun_w4_r3t.log | cut -c1-300
echo done
