# round 5 t2: RF kernel breakdown (rocprofv3 kernel stats)
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_rf -o rf -- python3 benchmarks/bench_configs.py rf > gpurun_out/r5/prof_rf.log 2>&1
echo "rc=$?"
