#!/bin/bash
# round 6: -factors 8 with KEEP (A/B vs KEEP 0), the N>1 wire: fp32 shard mean vs bf16 deltas
# (gloo rehearsal, 2 ranks on one card, same stream), non-general learners on the seq engine
set -o pipefail
O=gpurun_out/r6k
mkdir -p $O
export HM_NO_AUTOBUILD=1
for rep in 1 2; do
  for v in 0 9; do
    HM_FFM_VARIANT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --alt-run 0 --factors 8 > $O/bench_k8_v${v}_r$rep.log 2>&1 || exit 1
  done
done
for wire in native bf16_delta; do
  HM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --alt-run 0 --mix-wire $wire > $O/rehearsal_w2_$wire.log 2>&1 || exit 2
done
timeout -k 10 500 python -u benchmarks/linear_seq_probe.py --rows 1000000 --waves 128,512 --spread 8 --shared 1 \
  --rules "train_pa1: ;train_logregr: ;train_perceptron: ;train_adagrad_rda: ;train_pa: " \
  > $O/linear_seq_nongeneral.jsonl 2> $O/linear_seq_nongeneral.err || exit 3
echo ok
