#!/bin/bash
# Round-4 final re-validation at HEAD (after the last-level finalize change).
# kernel stats of the bench.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5y
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || true
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
tail -1 $O/bench.log | cut -c1-200
timeout -k 10 600 python -u benchmarks/bench_configs.py > $O/configs.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- \
  python3 bench.py --steps 20 --warmup 3 > $O/prof_bench.log 2>&1
