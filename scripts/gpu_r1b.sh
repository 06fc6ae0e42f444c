#!/bin/bash
# GPU call: kernel tests, smoke, FFM layout A/B, headline bench, rocprofv3 kernel stats.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python -u benchmarks/ffm_layout_ab.py > gpurun_out/ffm_layout_ab.log 2>&1
HM_FFM_MINW=6 timeout -k 10 300 python -u benchmarks/ffm_layout_ab.py --states bf16 --layouts packed > gpurun_out/ffm_layout_ab_minw6.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
timeout -k 10 300 python -u bench.py --layout split > gpurun_out/bench_split.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof.log 2>&1
echo done
