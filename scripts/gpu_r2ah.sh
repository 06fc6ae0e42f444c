#!/bin/bash
# Explicit MF: plain-store Hogwild vs atomic delta adds (fixture + ML-20M-shaped curves); MF GPU tests
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 400 python -u benchmarks/mf_atomic_probe.py fixture ml20m > gpurun_out/mf_atomic_probe_r2ah.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_mf.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_mf_r2ah.log 2>&1
echo done
