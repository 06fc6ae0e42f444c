#!/bin/bash
# round 6: BPR 4-factors-per-lane form at k = 16 / 32 too (vs the one-factor-per-lane forms, variant 5)
set -o pipefail
O=gpurun_out/r6ap
mkdir -p $O
export HM_NO_AUTOBUILD=1
for k in 16 32 10; do for v in 0 5; do
  HM_BPR_VARIANT=$v timeout -k 10 300 python -c "
import json, sys; sys.path.insert(0, '.')
from benchmarks.bench_configs import bench_bprmf
print(json.dumps(bench_bprmf(k=$k)))" > $O/bpr_k${k}_v$v.log 2>&1 || { tail -5 $O/bpr_k${k}_v$v.log; exit 1; }
  echo "k$k v$v $(tail -1 $O/bpr_k${k}_v$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['triples_per_s'], d['sampled_auc'])")"
done; done
timeout -k 10 400 python -u -m pytest tests/test_mf.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_mf.log 2>&1; rc=$?
grep FAILED $O/pytest_mf.log | head; tail -1 $O/pytest_mf.log
[ $rc -eq 0 ] || exit 2
echo ok
