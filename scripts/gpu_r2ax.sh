#!/bin/bash
# Round-2 last health run (final tree state)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_r2ax.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_gpu_r2ax.log
grep -q "Fatal\|core dumped\|Timeout" gpurun_out/pytest_gpu_r2ax.log && exit 3
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r2ax.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r2ax.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2ax -o run -- \
  python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_r2ax.log 2>&1
echo done
