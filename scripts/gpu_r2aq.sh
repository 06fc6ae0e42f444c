#!/bin/bash
# FM dense MFMA kernel: |V|^2 from the operand registers (no per-block V reloads); numerics + A/B
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 300 python -u -m pytest tests/test_fm.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fm_r2aq.log 2>&1
timeout -k 10 400 python -u benchmarks/probes/fm_dense_probe.py --ab --batches 8192,65536 --blocks 0,128 > gpurun_out/fm_dense_ab_r2aq.log 2>&1
echo done
