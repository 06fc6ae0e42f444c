#!/bin/bash
# round 6: side-table launch grid for the bf16 kernel (3 blocks per CU = 768 resident: 2,048
# blocks leave the last round 2/3 full) -- bench 20 / 5 at grids 1536 / 2304 / 2048 / 3072, x2
set -o pipefail
O=gpurun_out/r6ba
mkdir -p $O
export HM_NO_AUTOBUILD=1
for g in 1536 2304 2048 3072 1536 2304 2048 3072; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --grid $g > $O/g$g.json 2> $O/g$g.err || exit 2
  python -c "import json; d=json.load(open('$O/g$g.json')); print('grid $g', d['value'], d['logloss_gap'], d['value_bf16_state'], d['logloss_gap_bf16'])"
done
echo ok
