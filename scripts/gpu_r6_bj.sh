#!/bin/bash
# round 6 end: 2-rank rehearsal (gloo, both ranks on cuda:0) of the BASELINE configs 4 / 5 harness
# with the current tree (BPR's power-of-two grid) and of bench.py at N = 2 (self-launch form)
set -o pipefail
O=gpurun_out/r6bj
mkdir -p $O
export HM_NO_AUTOBUILD=1 HM_DIST_BACKEND=gloo
timeout -k 10 600 python -u benchmarks/bench_configs.py --gpus 2 gbdt rf bprmf > $O/configs_w2.log 2>&1 || { tail -20 $O/configs_w2.log; exit 1; }
grep '^{' $O/configs_w2.log | cut -c1-300
timeout -k 10 400 python -u bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_w2.log 2>&1 || { tail -20 $O/bench_w2.log; exit 2; }
grep '"metric"' $O/bench_w2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('w2', d['value'], d['config']['parallelism'], d['config']['linear_steps'], d.get('logloss_gap'), d.get('logloss_gap_bf16'))"
echo ok
