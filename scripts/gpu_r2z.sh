#!/bin/bash
# Round 2 call z: FFM sink variant with the pre-DMA store drain: semantics probe (grid 1 / full
# grid, with and without the linear term), FFM GPU tests, same-box A/B vs variant 3.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
TAG="${TAG:-r2z}"
timeout -k 10 400 python -u benchmarks/probes/ffm_sink_probe.py > gpurun_out/ffm_sink_probe_$TAG.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_$TAG.log
grep -q "Fatal\|core dumped\|Timeout\|rc=" gpurun_out/pytest_$TAG.log && exit 3
for rep in 1 2 3; do
  for v in 0 3 4; do
    echo "== variant $v rep $rep" >> gpurun_out/ffm_ab_$TAG.log
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py >> gpurun_out/ffm_ab_$TAG.log 2>&1
  done
done
echo done
