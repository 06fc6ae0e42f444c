#!/bin/bash
# round 6 validation: the full GPU suite (KEEP default in both pipelined FFM kernels, seq linear
# engine routing, pipelined mixing, BPR pf3), smoke, the driver's bench
set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 3
tail -1 $O/bench.log | cut -c1-400
