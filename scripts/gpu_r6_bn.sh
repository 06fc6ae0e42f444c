#!/bin/bash
# round 6: GBDT one-pass histogram grid below one block per CU (fewer image flushes onto the same
# addresses, some CUs idle): 256 / 224 / 192 / 128 blocks (x2)
set -o pipefail
O=gpurun_out/r6bn
mkdir -p $O
export HM_NO_AUTOBUILD=1
for b in 256 224 192 128 256 224 192 128; do
  HM_HIST_WIDE_BLOCKS=$b timeout -k 10 300 python benchmarks/bench_configs.py gbdt > $O/gbdt_$b.jsonl 2> $O/gbdt_$b.err || { tail -5 $O/gbdt_$b.err; exit 1; }
  echo "blocks $b $(cut -c1-300 $O/gbdt_$b.jsonl | grep -o '"ms_per_tree": [0-9.]*, "row_trees_per_s": [0-9]*, "test_auc": [0-9.]*')"
done
echo ok
