#!/bin/bash
# Full GPU suite, smoke, 1-GPU bench; the linear shared engine after the row-ahead prefetch.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5c
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || true
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
tail -1 $O/bench.log | cut -c1-200
timeout -k 10 600 python -u benchmarks/linear_rules_parity.py 1000000 "-opt adagrad" "-opt adam -eta0 0.01" \
  "-opt sgd -eta0 0.05" "-opt adagrad -reg l1 -lambda 1e-6" > $O/linear_prefetch.jsonl 2>&1
timeout -k 10 300 python -u benchmarks/bench_configs.py linear_hashed > $O/linear_hashed.log 2>&1
