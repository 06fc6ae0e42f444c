#!/bin/bash
# Round 3: every BASELINE config re-measured on one MI355X (bench_configs.py), then a rocprofv3
# --kernel-trace --stats run per GPU config (per-kernel device time next to each number).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/configs_r3
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u benchmarks/bench_configs.py linear_gpu linear_hashed fm gbdt xgboost bprmf > gpurun_out/configs_r3/bench_configs_r3.jsonl 2>gpurun_out/configs_r3/bench_configs_r3.err
timeout -k 10 300 python -u benchmarks/bench_configs.py rf >> gpurun_out/configs_r3/bench_configs_r3.jsonl 2>>gpurun_out/configs_r3/bench_configs_r3.err
cat gpurun_out/configs_r3/bench_configs_r3.jsonl | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for c in linear_hashed fm gbdt bprmf; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/configs_r3/prof_$c -o run -- \
    python3 benchmarks/bench_configs.py $c > gpurun_out/configs_r3/prof_$c.log 2>&1
  echo "prof $c ok"
done
echo done
