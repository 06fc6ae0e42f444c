#!/bin/bash
# Round 4, first GPU call: fresh-box bench (autobuild left ON: the library must not recompile),
# the GPU suite, then a rocprofv3 kernel profile of the bench.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
cat $O/bench.log | tail -1
export HM_NO_AUTOBUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || true
tail -5 $O/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1
find $O/prof -name '*stats*'
bash scripts/gpu_r4b.sh
bash scripts/gpu_r4c.sh
bash scripts/gpu_r4d.sh
