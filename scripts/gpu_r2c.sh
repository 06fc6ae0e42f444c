#!/bin/bash
# Round 2 call c: lean FFM kernel — GPU tests, smoke, same-box interleaved A/B against the
# round-1 ffm_packed_kernel (HM_FFM_VARIANT=1), bf16 and fp32 state.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2c}"
timeout -k 10 300 python -u -m pytest tests/test_ffm.py tests/test_mix_lowp.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
for rep in 1 2; do
  for v in 1 0; do
    for st in bf16 fp32; do
      echo "== variant $v state $st rep $rep" >> gpurun_out/ffm_ab_$TAG.log
      HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py --state $st >> gpurun_out/ffm_ab_$TAG.log 2>&1
    done
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_$TAG.log 2>&1
echo done
