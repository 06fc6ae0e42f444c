#!/bin/bash
# FFM fp32-state pipelined kernel (A/B vs the lean kernel), bf16 unchanged; MF line-padded bias atomics
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 400 python -u -m pytest tests/test_mf.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_r2ak.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_r2ak.log
grep -q "Fatal\|core dumped\|Timeout\|rc=" gpurun_out/pytest_r2ak.log && exit 3
HM_FFM_VARIANT=2 timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r2ak.log 2>&1
for rep in 1 2; do
  for v in 0 2; do
    echo "== fp32 variant $v rep $rep" >> gpurun_out/ffm_fp32_ab_r2ak.log
    HM_FFM_VARIANT=$v timeout -k 10 300 python -u bench.py --state fp32 >> gpurun_out/ffm_fp32_ab_r2ak.log 2>&1
  done
done
echo "== bf16 default" >> gpurun_out/ffm_fp32_ab_r2ak.log
timeout -k 10 300 python -u bench.py >> gpurun_out/ffm_fp32_ab_r2ak.log 2>&1
timeout -k 10 300 python -u benchmarks/mf_contention_probe.py > gpurun_out/mf_contention_r2ak.log 2>&1
timeout -k 10 400 python -u benchmarks/mf_atomic_probe.py ml20m > gpurun_out/mf_atomic_probe_r2ak.log 2>&1
echo done
