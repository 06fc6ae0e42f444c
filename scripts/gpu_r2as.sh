#!/bin/bash
# RandomForest kernel breakdown (rocprofv3 kernel trace) + wall time per tree
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1 PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
timeout -k 10 200 python -u benchmarks/probes/rf_prof_target.py 10 > gpurun_out/rf_wall_r2as.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rf -o run -- \
  python3 benchmarks/probes/rf_prof_target.py 10 > gpurun_out/prof_rf.log 2>&1
echo done
