#!/bin/bash
# Round 2 call d: LDS-DMA pipelined FFM kernel — GPU tests, smoke, same-box interleaved A/B of
# variants 0 (pipe) / 2 (lean) / 1 (round-1 packed), then counters of the pipe kernel.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2d}"
timeout -k 10 300 python -u -m pytest tests/test_ffm.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
for rep in 1 2; do
  for v in 1 2 0; do
    echo "== variant $v state bf16 rep $rep" >> gpurun_out/ffm_ab_$TAG.log
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py >> gpurun_out/ffm_ab_$TAG.log 2>&1
  done
done
OUT=ffm_pmc_pipe PAT=ffm_pipe bash scripts/ffm_counters.sh
echo done
