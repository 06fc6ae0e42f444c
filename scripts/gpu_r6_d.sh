#!/bin/bash
# round 6: seq engine at 512 / 1024 rows in flight on a second data seed (+ AdaGrad rules vs the
# shared engine), FM write-through (SC1) store variants at grid 256 / 128, the mix probe after the
# fused unpack + 32-bit view indexing
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 400 python -u benchmarks/linear_seq_probe.py --rows 1000000 --waves 512,1024 --spread 8 --seed 11 \
  --rules "-opt adam -eta0 0.01;-opt sgd -eta0 0.05;-opt rmsprop -eta0 0.01;-opt adadelta;-opt momentum -eta0 0.005;-opt eve -eta0 0.01;-opt adagrad;-opt adagrad -reg l1 -lambda 1e-6;-opt adagrad -reg no" \
  > $O/linear_seq_seed11.jsonl 2> $O/linear_seq_seed11.err || exit 1
PROBE_VARIANTS=0,2,3 PROBE_REPS=2 timeout -k 10 400 python -u benchmarks/fm_grid_parity_probe.py 256 128 > $O/fm_wt_parity.jsonl 2> $O/fm_wt_parity.err || exit 2
timeout -k 10 200 python -u benchmarks/mix_pipe_probe.py --bits 20 --reps 10 --buckets 0,32,64,128 > $O/mix_pipe_probe.jsonl 2> $O/mix_pipe_probe.err || exit 3
echo ok
