#!/bin/bash
# Hot-feature flush schedule adapted to the pass length: the 2^24 parity test (200 K rows, one
# epoch) and the 1 M-row parity bench for the hot rules.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4t
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_linear.py \
  -k "hashed_2p24" > $O/pytest_2p24.log 2>&1 || true
grep -E "PASSED|FAILED|AssertionError: \{" $O/pytest_2p24.log | tail -40
timeout -k 10 600 python -u benchmarks/linear_rules_parity.py 1000000 "-opt adagrad" "-opt adagrad -reg no" \
  "-opt adagrad -reg l1 -lambda 1e-6" "-opt adadelta" > $O/parity_1m.jsonl 2>&1
timeout -k 10 300 python -u benchmarks/bench_configs.py linear_hashed > $O/bench_linear_hashed.log 2>&1
