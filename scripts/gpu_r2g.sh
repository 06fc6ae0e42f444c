#!/bin/bash
# Round 2 call g: pipe kernel v3 (meta + linear state by LDS-DMA, line-padded feature blocks,
# whole-line writes) — tests, smoke, same-box A/B, counters.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2g}"
timeout -k 10 300 python -u -m pytest tests/test_ffm.py tests/test_mix_lowp.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
for rep in 1 2; do
  for v in 1 2 0; do
    echo "== variant $v state bf16 rep $rep" >> gpurun_out/ffm_ab_$TAG.log
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py >> gpurun_out/ffm_ab_$TAG.log 2>&1
  done
done
echo "== variant 0 state fp32" >> gpurun_out/ffm_ab_$TAG.log
timeout -k 10 300 python -u bench.py --state fp32 >> gpurun_out/ffm_ab_$TAG.log 2>&1
OUT=ffm_pmc_pipe3 PAT=ffm_pipe bash scripts/ffm_counters.sh
echo done
