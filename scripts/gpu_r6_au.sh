#!/bin/bash
# round 6: bench.py's N = 8 path rehearsed with 8 gloo ranks sharing cuda:0 (side-table linear
# mode, bucketed pipelined mix); rows/s meaningless, held-out logloss and the JSON line checked
set -o pipefail
O=gpurun_out/r6au
mkdir -p $O
export HM_NO_AUTOBUILD=1 HM_DIST_BACKEND=gloo
env $EXTRA timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 8 --steps 12 --warmup 3 > $O/rehearsal_w8.log 2>&1 || { tail -30 $O/rehearsal_w8.log; exit 1; }
grep '"metric"' $O/rehearsal_w8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('n_gpus','world','value','logloss_heldout','logloss_heldout_bf16','rows_trained_per_rank','dist_backend')})"
echo ok
