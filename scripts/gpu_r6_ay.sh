#!/bin/bash
# round 6: the N > 1 wire at bench scale: fp32 replicas mixing bf16 deltas (default) vs the fp32
# model itself (--mix-wire native), gloo rehearsals of N = 8 and N = 2 ranks on cuda:0, 20 / 5 stream
set -o pipefail
O=gpurun_out/r6ay
mkdir -p $O
export HM_NO_AUTOBUILD=1 HM_DIST_BACKEND=gloo
run() {  # n, wire
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 \
    --master-port 2955$1 bench.py --gpus $1 --steps 20 --warmup 5 --mix-wire $2 > $O/w$1_$2.log 2>&1 || { tail -30 $O/w$1_$2.log; exit 1; }
  grep '"metric"' $O/w$1_$2.log > $O/w$1_$2.json
  python -c "import json; d=json.load(open('$O/w$1_$2.json')); print('w$1 $2', {k: d.get(k) for k in ('logloss_heldout','logloss_gap','logloss_heldout_bf16','logloss_gap_bf16')}, d['config'].get('mix_wire'), d['config'].get('mixed_bytes_per_mix'))"
}
run 8 native && run 8 bf16_delta && run 2 native && run 2 bf16_delta && echo ok
