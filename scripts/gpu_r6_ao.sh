#!/bin/bash
# round 6: BPR at k = 64 with 16 lanes x 4 factors per triple (16-B loads / stores, four triples
# per wave instruction; default) vs the 64-lane form (HM_BPR_VARIANT=5), interleaved; BPR tests
set -o pipefail
O=gpurun_out/r6ao
mkdir -p $O
export HM_NO_AUTOBUILD=1
for rep in 1 2; do for v in 0 5; do
  HM_BPR_VARIANT=$v timeout -k 10 300 python benchmarks/bench_configs.py bprmf > $O/bpr_v${v}_$rep.log 2>&1 || { tail -5 $O/bpr_v${v}_$rep.log; exit 1; }
  echo "v$v $(tail -1 $O/bpr_v${v}_$rep.log | cut -c1-260)"
done; done
timeout -k 10 400 python -u -m pytest tests/test_mf.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_mf.log 2>&1; rc=$?
grep FAILED $O/pytest_mf.log | head; tail -1 $O/pytest_mf.log
[ $rc -eq 0 ] || exit 2
echo ok
