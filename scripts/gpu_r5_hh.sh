# round 5 hh: kernel stats of the -w0 probe
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_w0 -o w0 -- python3 benchmarks/ffm_w0_rate_probe.py > gpurun_out/r5/prof_w0.log 2>&1
echo "rc=$?"
