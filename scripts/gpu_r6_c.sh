#!/bin/bash
# round 6: seq-engine rows-in-flight sweep on one XCD (all non-AdaGrad general rules, 2 seeds),
# the mix probe's kernel trace, and the generic FFM kernel's linear-record probe
set -o pipefail
O=gpurun_out/r6c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u benchmarks/linear_seq_probe.py --rows 1000000 --waves 128,256,512 --spread 8 --shared 0 \
  --rules "-opt adam -eta0 0.01;-opt sgd -eta0 0.05;-opt rmsprop -eta0 0.01;-opt adadelta;-opt momentum -eta0 0.005;-opt nesterov -eta0 0.005;-opt nadam -eta0 0.01;-opt adamhd -eta0 0.01;-opt rmspropgraves -eta0 0.001;-opt eve -eta0 0.01" \
  > $O/linear_seq_sweep.jsonl 2> $O/linear_seq_sweep.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_mix -o mix -- python benchmarks/mix_pipe_probe.py --bits 20 --reps 5 --buckets 0,64 > $O/mix_prof.log 2>&1 || exit 2
timeout -k 10 300 python -u benchmarks/ffm_generic_lin_probe.py --reps 2 > $O/generic_lin_records.jsonl 2> $O/generic_lin.err || exit 3
timeout -k 10 300 python -u benchmarks/ffm_generic_lin_probe.py --reps 2 --separate > $O/generic_lin_separate.jsonl 2>> $O/generic_lin.err || exit 4
echo ok
