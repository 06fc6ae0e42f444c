#!/bin/bash
# The 2^24 per-rule parity test after restricting owner mode to AdaGrad-L1 / elastic net, next
# to the parity bench at the test's 200 K rows.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4r
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_linear.py \
  -k "hashed_2p24" > $O/pytest_2p24.log 2>&1 || true
tail -20 $O/pytest_2p24.log
timeout -k 10 600 python -u benchmarks/linear_rules_parity.py 200000 "-opt adagrad -reg no" "-opt sgd -eta0 0.05" \
  "-opt adam -eta0 0.01" "-opt adadelta" > $O/parity_200k.jsonl 2>&1
timeout -k 10 300 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_fm.py \
  tests/test_mix_rccl.py > $O/pytest_fm_rccl.log 2>&1 || true
tail -5 $O/pytest_fm_rccl.log
