#!/bin/bash
# round 6: BPR grid rounded up to a power of two (852 -> 1,024 blocks on ML-20M shape): MF / BPR
# GPU tests, config 5 x2
set -o pipefail
O=gpurun_out/r6bg
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_mf.py tests/test_topic_recommend.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_mf.log 2>&1 || { grep -E "FAILED|Error" $O/pytest_mf.log | head; tail -3 $O/pytest_mf.log; exit 1; }
tail -1 $O/pytest_mf.log
for i in 1 2; do
  timeout -k 10 300 python benchmarks/bench_configs.py bprmf > $O/bpr$i.jsonl 2> $O/bpr$i.err || exit 2
  cut -c1-400 $O/bpr$i.jsonl
done
echo ok
