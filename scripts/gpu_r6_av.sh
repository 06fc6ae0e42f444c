#!/bin/bash
# round 6: the N = 8 gloo rehearsal's bf16 model (0.512 with the side table) with plain linear
# stores, and with the side table but no dp step scaling, to isolate it
set -o pipefail
O=gpurun_out/r6av
mkdir -p $O
export HM_NO_AUTOBUILD=1 HM_DIST_BACKEND=gloo
run() {  # tag, env / args
  local tag=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29542 bench.py --gpus 8 --steps 12 --warmup 3 "$@" > $O/w8_$tag.log 2>&1 || { tail -30 $O/w8_$tag.log; exit 1; }
  grep '"metric"' $O/w8_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', {k: d.get(k) for k in ('logloss_heldout','logloss_heldout_bf16','mix_wire')})"
}
run plain "HM_FFM_LIN_ATOMIC=0"
run side_p05 "HM_FFM_LIN_ATOMIC=4" --dp-lr-power 0.5
echo ok
