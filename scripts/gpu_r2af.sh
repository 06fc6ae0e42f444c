#!/bin/bash
# Round-2 re-entry health run: GPU tests, smoke, bench, rocprofv3 kernel stats.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r2af.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r2af.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r2af.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2af -o run -- \
  python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_r2af.log 2>&1
echo done
