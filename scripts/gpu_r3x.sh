#!/bin/bash
# Round 3: native touched-mask kernel (util.hip) — FM/FFM GPU tests, then the FM config (whose
# timed epoch carried ~10 ms of torch bookkeeping per 2 M rows) baseline library vs new.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 500 python -u -m pytest tests/test_fm.py tests/test_ffm.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3x_pytest_fm_ffm.log 2>&1
tail -2 gpurun_out/r3x_pytest_fm_ffm.log
for rep in 1 2; do
  timeout -k 10 300 python -u benchmarks/bench_configs.py fm >> gpurun_out/r3x_fm.log 2>&1
done
grep '^{' gpurun_out/r3x_fm.log | cut -c1-250
echo done
