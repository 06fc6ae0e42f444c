# round 5 ff: fp32 FFM kernel rate with / without the global bias
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 200 python -u benchmarks/ffm_w0_rate_probe.py > gpurun_out/r5/ffm_w0_rate.jsonl 2> gpurun_out/r5/ffm_w0_rate.err
echo "rc=$?"
