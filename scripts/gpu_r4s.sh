#!/bin/bash
# AdaGrad hot flush with the returning accumulator add; the parity test's setup vs the bench's.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4s
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u benchmarks/linear_parity_debug.py "-opt adagrad -reg no" "-opt adagrad -reg l2 -lambda 1e-6" \
  "-opt adagrad" "-opt sgd -eta0 0.05" "-opt adam -eta0 0.01" "-opt adadelta" > $O/debug.jsonl 2>&1
timeout -k 10 600 python -u benchmarks/linear_rules_parity.py 1000000 "-opt adagrad -reg no" "-opt adagrad -reg l2 -lambda 1e-6" \
  "-opt adagrad" > $O/parity_adagrad_1m.jsonl 2>&1
