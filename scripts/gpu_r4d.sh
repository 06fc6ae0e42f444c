#!/bin/bash
# Same-box A/B: FM gather-prefetch kernel (HM_FM_VARIANT=2) vs fm_pipe_kernel (0); BPR pipelined
# bitmap sampler (HM_BPR_VARIANT=0) vs bpr_kernel (1); then the FM / MF GPU tests on the new ones.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4d
mkdir -p $O
export HM_NO_AUTOBUILD=1
for rep in 1 2; do
  for v in 0 2; do
    echo "== fm variant $v rep $rep" >> $O/ab.log
    HM_FM_VARIANT=$v timeout -k 10 300 python -u benchmarks/bench_configs.py fm >> $O/ab.log 2>&1
  done
  for v in 1 0; do
    echo "== bpr variant $v rep $rep" >> $O/ab.log
    HM_BPR_VARIANT=$v timeout -k 10 300 python -u benchmarks/bench_configs.py bprmf >> $O/ab.log 2>&1
  done
done
HM_FM_VARIANT=2 timeout -k 10 600 python -u -m pytest tests/test_fm.py tests/test_mf.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_fm_mf.log 2>&1 || true
tail -3 $O/pytest_fm_mf.log
