#!/bin/bash
# round 6: FM hot-feature write-through (threshold sweep, parity at grid 256 / 128 + config-2 rate),
# seq-engine rows-in-flight on 3 seeds, generic FFM kernel with 16-B record updates
set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
PROBE_HOT=0,0.01,0.002 PROBE_REPS=2 timeout -k 10 400 python -u benchmarks/fm_grid_parity_probe.py 256 128 > $O/fm_hot_parity.jsonl 2> $O/fm_hot_parity.err || exit 1
for h in 0 0.01 0.002; do for g in 256 128; do
  HM_FM_HOT_FRAC=$h HM_BENCH_FM_OPTS="-grid $g" timeout -k 10 200 python benchmarks/bench_configs.py fm > $O/fm_rate_h${h}_g${g}.log 2>&1 || exit 2
done; done
for seed in 5 11 23; do
  timeout -k 10 400 python -u benchmarks/linear_seq_probe.py --rows 1000000 --waves 128,256,512 --spread 8 --seed $seed --shared 0 \
    --rules "-opt adam -eta0 0.01;-opt sgd -eta0 0.05;-opt rmsprop -eta0 0.01;-opt adadelta;-opt momentum -eta0 0.005" \
    > $O/linear_seq_s$seed.jsonl 2> $O/linear_seq_s$seed.err || exit 3
done
timeout -k 10 300 python -u benchmarks/ffm_generic_lin_probe.py --reps 2 --variants 1 > $O/generic_lin_rec16.jsonl 2> $O/generic_lin.err || exit 4
HM_FFM_LPACK=0 timeout -k 10 300 python -u benchmarks/ffm_generic_lin_probe.py --reps 2 --variants 1 > $O/generic_lin_rec4.jsonl 2>> $O/generic_lin.err || exit 5
echo ok
