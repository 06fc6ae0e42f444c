#!/bin/bash
# round 6: N = 8 gloo rehearsal (8 ranks on cuda:0) on the driver's 20 / 5 stream (pinned N = 8
# sequential reference 0.437804): side-table vs plain linear stores, FTRL alpha's dp power
set -o pipefail
O=gpurun_out/r6aw
mkdir -p $O
export HM_NO_AUTOBUILD=1 HM_DIST_BACKEND=gloo
run() {  # tag, env
  local tag=$1; shift
  env $1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29543 bench.py --gpus 8 --steps 20 --warmup 5 > $O/w8_$tag.log 2>&1 || { tail -30 $O/w8_$tag.log; exit 1; }
  grep '"metric"' $O/w8_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', {k: d.get(k) for k in ('logloss_heldout','logloss_gap','logloss_heldout_bf16','logloss_gap_bf16')})"
}
run plain "HM_FFM_LIN_ATOMIC=0"
run side "HM_FFM_LIN_ATOMIC=4"
run side_a0 "HM_FFM_DP_ALPHA_POWER=0"
run side_a05 "HM_FFM_DP_ALPHA_POWER=0.5"
echo ok
