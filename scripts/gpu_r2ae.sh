#!/bin/bash
# FFM corrected A/B: pipe vmcnt (0, default) vs polled early (5) / late (4) vs round-1 packed (1);
# grid-1 semantics probe; FFM GPU tests
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_r2ae.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_r2ae.log
grep -q "Fatal\|core dumped\|Timeout\|rc=" gpurun_out/pytest_r2ae.log && exit 3
for rep in 1 2 3; do
  for v in 0 5 4 1; do
    echo "== variant $v rep $rep" >> gpurun_out/ffm_ab_r2ae.log
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py >> gpurun_out/ffm_ab_r2ae.log 2>&1
  done
done
timeout -k 10 500 python -u benchmarks/probes/ffm_sink_probe.py > gpurun_out/ffm_sink_probe_r2ae.log 2>&1
echo done
