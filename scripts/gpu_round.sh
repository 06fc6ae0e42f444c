#!/bin/bash
# One gpurun call: GPU tests, smoke, a short bench and a rocprofv3 kernel profile.
# Every GPU step has its own time limit; the first failure ends the script.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
STEPS="${STEPS:-tests smoke bench prof configs}"
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/pytest_gpu.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee gpurun_out/smoke.log ;;
    bench) timeout -k 10 300 python bench.py ${BENCH_ARGS:-} 2>&1 | tee gpurun_out/bench.log ;;
    prof)  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
           timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
             python3 bench.py --steps 10 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
           find gpurun_out/prof -name '*stats*' ;;
    configs) timeout -k 10 600 python benchmarks/bench_configs.py linear_gpu fm gbdt bprmf > gpurun_out/configs.log 2>&1
             timeout -k 10 300 python benchmarks/bench_configs.py rf >> gpurun_out/configs.log 2>&1 ;;
    *) timeout -k 10 600 bash -c "$s" ;;
  esac
done
