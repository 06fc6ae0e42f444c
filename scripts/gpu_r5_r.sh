# round 5 r: spread of train_fm's Hogwild gap past 2^20 rows by grid
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u benchmarks/fm_grid_parity_probe.py 32 64 128 256 > gpurun_out/r5/fm_grid_parity_probe.jsonl 2> gpurun_out/r5/fm_grid_parity_probe.err
echo "rc=$?"
