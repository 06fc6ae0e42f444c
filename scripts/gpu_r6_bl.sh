#!/bin/bash
# round 6: fp32 side-table launch grid vs the gap margin (2,048 = 4 full rounds of 512 resident;
# more blocks flush sooner): bench 20 / 5 at 2,048 / 2,560 / 3,072 / 4,096 blocks, x2 (fp32 numbers)
set -o pipefail
O=gpurun_out/r6bl
mkdir -p $O
export HM_NO_AUTOBUILD=1
for g in 2048 2560 3072 4096 2048 2560 3072 4096; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --grid $g > $O/g$g.json 2> $O/g$g.err || exit 2
  python -c "import json; d=json.load(open('$O/g$g.json')); print('grid $g', d['value'], d['logloss_gap'], d['value_bf16_state'], d['logloss_gap_bf16'])"
done
echo ok
