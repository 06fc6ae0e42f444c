#!/bin/bash
# Round 3: 3-level view pack / fused merge+pack kernels for the overlapped mix; probe again.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_mix_lowp.py -m gpu -x -v --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r3m_pytest_mix.log
timeout -k 10 200 python benchmarks/mix_overlap_probe.py --world 8 2>&1 | tee gpurun_out/r3m_mix_overlap_w8.log
timeout -k 10 200 python benchmarks/mix_overlap_probe.py --world 8 --state fp32 2>&1 | tee gpurun_out/r3m_mix_overlap_w8_fp32.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mixprof2 -o run -- python3 benchmarks/mix_overlap_probe.py --world 8 > gpurun_out/r3m_mixprof.log 2>&1
