#!/bin/bash
# round 6: bench with the pinned sequential reference, the row-order experiment, the pipelined
# mix (bit-identity test + device ms per mix), the near-sequential linear engine's sweep
set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_mix_rccl.py > $O/pytest_mix.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_default.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --row-order spread > $O/bench_spread.log 2>&1 || exit 3
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_default2.log 2>&1 || exit 4
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --row-order spread > $O/bench_spread2.log 2>&1 || exit 5
timeout -k 10 200 python -u benchmarks/mix_pipe_probe.py --bits 20 --reps 10 --buckets 0,16,32,64 > $O/mix_pipe_probe.jsonl 2> $O/mix_pipe_probe.err || exit 6
timeout -k 10 400 python -u benchmarks/linear_seq_probe.py --rows 1000000 --waves 8,16,32,64,128 --spread 8,1 > $O/linear_seq_probe.jsonl 2> $O/linear_seq_probe.err || exit 7
echo ok
