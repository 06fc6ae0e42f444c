#!/bin/bash
# Fused MFMA top-k: GPU tests + bench (+ optional rocprofv3 kernel stats).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-x}"
timeout -k 10 300 python -u -m pytest tests/test_topk_mips.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_mips_$TAG.log 2>&1
timeout -k 10 300 python -u benchmarks/mips_bench.py ${MIPS_ARGS:-} > gpurun_out/mips_bench_$TAG.log 2>&1
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mips_prof_$TAG -o run -- python3 benchmarks/mips_bench.py --reps 3 > gpurun_out/mips_prof_$TAG.log 2>&1
fi
echo done
