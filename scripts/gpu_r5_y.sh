# round 5 y: train_fm hot-feature atomics (where the Hogwild gap lives)
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u benchmarks/fm_hot_probe.py 0 32 512 8192 65536 > gpurun_out/r5/fm_hot_probe.jsonl 2> gpurun_out/r5/fm_hot_probe.err
echo "rc=$?"
