#!/bin/bash
# Round 3: hot-feature pre-aggregation in the shared linear kernel (probe), bench-scale parity
# variance (3 runs of bench.py --gen-device cpu).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 400 python benchmarks/linear_hot_probe.py 2>&1 | tee gpurun_out/linear_hot_probe.log
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --gen-device cpu 2>&1 | tee gpurun_out/r3n_cpugen_$rep.log
done
