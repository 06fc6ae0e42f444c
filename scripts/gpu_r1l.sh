#!/bin/bash
# Round health of the rebuilt tree (fresh container): full GPU suite, smoke, bench and
# rocprofv3 kernel stats of the headline bench.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_l.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_l.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_l.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_l -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_l.log 2>&1
echo done
