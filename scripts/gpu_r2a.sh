#!/bin/bash
# Round-2 health of the restored tree: full GPU suite, smoke, bench (bf16 and fp32 state) and
# rocprofv3 kernel stats of the headline bench.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2a}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --state fp32 ${BENCH_ARGS:-} >> gpurun_out/bench_$TAG.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/prof_$TAG.log 2>&1
echo done
