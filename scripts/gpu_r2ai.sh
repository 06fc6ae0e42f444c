#!/bin/bash
# FM MFMA gradient kernel numerics + A/B; explicit MF atomic modes (items-only hybrid)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 300 python -u -m pytest tests/test_fm.py tests/test_mf.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fm_mf_r2ai.log 2>&1 || echo "pytest rc=$?"
grep -q "Fatal\|core dumped\|Timeout" gpurun_out/pytest_fm_mf_r2ai.log && exit 3
timeout -k 10 400 python -u benchmarks/probes/fm_dense_probe.py --ab --batches 8192,65536 > gpurun_out/fm_dense_ab_r2ai.log 2>&1
timeout -k 10 400 python -u benchmarks/mf_atomic_probe.py fixture ml20m > gpurun_out/mf_atomic_probe_r2ai.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fmd -o run -- \
  python3 benchmarks/probes/fm_dense_probe.py --ab --batches 65536 --blocks 0 --rows 2000000 > gpurun_out/prof_fmd.log 2>&1
echo done
