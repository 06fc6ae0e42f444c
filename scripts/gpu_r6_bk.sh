#!/bin/bash
# round 6 final-tree validation (BPR power-of-two grid on top of val5): whole GPU suite, smoke, the driver's bench, the other BASELINE configs
# (FM config 2, BPR config 5 on one card, GBDT, RF), kernel stats of the driver's bench
set -o pipefail
O=gpurun_out/r6bk
mkdir -p $O
export HM_NO_AUTOBUILD=1 TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
grep -E "FAILED" $O/pytest_gpu.log | head -5; tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 3
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d.get('logloss_gap'), d.get('value_bf16_state'), d.get('logloss_gap_bf16'))"
timeout -k 10 600 python benchmarks/bench_configs.py fm bprmf gbdt rf > $O/configs.jsonl 2> $O/configs.err || { tail -5 $O/configs.err; exit 4; }
cut -c1-230 $O/configs.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/bench_prof.log 2>&1 || exit 5
echo ok
