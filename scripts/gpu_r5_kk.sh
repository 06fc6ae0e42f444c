# round 5 kk: train_ffm kernel rate under non-default options
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u benchmarks/ffm_option_rate_sweep.py > gpurun_out/r5/ffm_option_rate_sweep.jsonl 2> gpurun_out/r5/ffm_option_rate_sweep.err
echo "rc=$?"
timeout -k 10 300 python -u benchmarks/fm_option_rate_sweep.py > gpurun_out/r5/fm_option_rate_sweep.jsonl 2> gpurun_out/r5/fm_option_rate_sweep.err
echo "fm rc=$?"
