#!/bin/bash
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 200 python bench.py 2>&1 | tee gpurun_out/r3b_bench.log
timeout -k 10 200 python bench.py --adagrad element 2>&1 | tee gpurun_out/r3b_bench_elementwise.log
timeout -k 10 400 python benchmarks/ffm_hogwild_probe.py 2>&1 | tee gpurun_out/r3b_hogwild_probe.log
