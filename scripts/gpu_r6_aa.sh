#!/bin/bash
# round 6: multi-rank rehearsal of bench.py (2 and 4 gloo ranks sharing cuda:0) with the side-table
# linear mode, then the linear parity test at the new rmspropgraves routing
set -o pipefail
O=gpurun_out/r6aa
mkdir -p $O
export HM_NO_AUTOBUILD=1
for n in 2 4; do
  HM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 2953$n bench.py --gpus $n --steps 12 --warmup 3 > $O/rehearsal_w$n.log 2>&1 || { tail -20 $O/rehearsal_w$n.log; exit 1; }
  grep '"metric"' $O/rehearsal_w$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('w$n', d['value'], d.get('logloss_gap'), d.get('logloss_seq_ref'), d.get('world'))"
done
timeout -k 10 400 python -u -m pytest tests/test_linear.py -m gpu -v --timeout 300 --timeout-method thread -k "hashed_2p24_logloss_parity" > $O/pytest_linear.log 2>&1; tail -1 $O/pytest_linear.log
echo ok
