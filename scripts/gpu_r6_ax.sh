#!/bin/bash
# round 6: replicas that mix use the plain linear stores (dp_lin_mode): N = 8 and N = 2 gloo
# rehearsals on the 20 / 5 stream, N = 1 bench (side table)
set -o pipefail
O=gpurun_out/r6ax
mkdir -p $O
export HM_NO_AUTOBUILD=1
for n in 8 2; do
  HM_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 2954$n bench.py --gpus $n --steps 20 --warmup 5 > $O/w$n.log 2>&1 || { tail -30 $O/w$n.log; exit 1; }
  grep '"metric"' $O/w$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('w$n', {k: d.get(k) for k in ('logloss_heldout','logloss_gap','logloss_heldout_bf16','logloss_gap_bf16')})"
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_n1.log 2>&1 || exit 2
tail -1 $O/bench_n1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('n1', d['value'], d.get('logloss_gap'), d.get('value_bf16_state'), d.get('logloss_gap_bf16'))"
echo ok
