#!/bin/bash
# Round 2 call b: new mix kernels + smoke (kernel == CPU engine), MF L1-coherence A/B,
# hardware counters of the shipped ffm_packed_kernel.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_mix_lowp.py tests/test_mf.py tests/test_ffm.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_r2b.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r2b.log 2>&1
timeout -k 10 400 python -u benchmarks/mf_coherence_probe.py > gpurun_out/mf_coherence_r2b.log 2>&1
OUT=ffm_pmc_packed bash scripts/ffm_counters.sh
echo done
