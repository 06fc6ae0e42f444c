#!/bin/bash
# Round 2 call v: pipelined FM kernel — GPU tests, then same-box interleaved A/B against the
# previous kernel (HM_FM_VARIANT=1) on the config-2 bench.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2v}"
timeout -k 10 400 python -u -m pytest tests/test_fm.py tests/test_sql.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_$TAG.log
grep -q "Fatal\|core dumped\|Timeout\|rc=" gpurun_out/pytest_$TAG.log && exit 3
for rep in 1 2; do
  for v in 0 1; do
    echo "== variant $v rep $rep" >> gpurun_out/fm_ab_$TAG.log
    HM_FM_VARIANT=$v timeout -k 10 300 python -u benchmarks/bench_configs.py fm >> gpurun_out/fm_ab_$TAG.log 2>&1
  done
done
echo done
