#!/bin/bash
# round 6: GBDT's all-features histogram pass on 256 blocks of 1,024 threads = ONE block per CU
# although its 57 KB image would let two share a CU: grid sweep 256 / 512 / 768 / 1024 (x2)
set -o pipefail
O=gpurun_out/r6bh
mkdir -p $O
export HM_NO_AUTOBUILD=1
for b in 256 512 768 1024 256 512 768 1024; do
  HM_HIST_WIDE_BLOCKS=$b timeout -k 10 300 python benchmarks/bench_configs.py gbdt > $O/gbdt_$b.jsonl 2> $O/gbdt_$b.err || { tail -5 $O/gbdt_$b.err; exit 1; }
  echo "blocks $b $(cut -c1-300 $O/gbdt_$b.jsonl | grep -o '"ms_per_tree": [0-9.]*, "row_trees_per_s": [0-9]*, "test_auc": [0-9.]*')"
done
echo ok
