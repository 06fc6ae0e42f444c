#!/bin/bash
# (1) FFM same-stream parity with the coherent (SC1) loads/stores variant vs default;
# (2) per-rule rows-in-flight sweep of the linear shared engine at 2^24;
# (3) bench.py's real N-rank path rehearsed on one card (gloo) at N = 2, 4 vs one rank on
#     the same total rows (benchmarks/dp_parity.py).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4f
mkdir -p $O
export HM_NO_AUTOBUILD=1
for v in 0 7; do
  echo "== variant $v" >> $O/parity_coh.log
  HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py --gen-device cpu --mix-probe 0 >> $O/parity_coh.log 2>&1
done
echo "== variant 7 grid 32768" >> $O/parity_coh.log
HM_FFM_VARIANT=7 timeout -k 10 300 python -u bench.py --gen-device cpu --mix-probe 0 --grid 32768 >> $O/parity_coh.log 2>&1
HM_RULE_WAVES=512,128,32 timeout -k 10 900 python -u benchmarks/linear_rules_parity.py 1000000 \
  "-opt sgd -eta0 0.05" "-opt momentum -eta0 0.05" "-opt nesterov -eta0 0.05" "-opt adagrad -reg l1 -lambda 1e-6" \
  "-opt rmsprop" "-opt rmspropgraves" "-opt adadelta" "-opt adam" "-opt nadam" "-opt eve" "-opt adamhd" \
  > $O/linear_rules_waves.jsonl 2>&1
HM_DIST_BACKEND=gloo timeout -k 10 900 python -u benchmarks/dp_parity.py --worlds 2 4 --device cuda --steps 10 \
  --warmup 0 --batch 262144 --hash-bits 20 --eval-rows 262144 --same-steps 0 > $O/dp_parity_gloo.jsonl 2>&1
