#!/bin/bash
# FFM early-training gap vs the number of blocks (rows in flight) over the first 500 K rows
set -o pipefail
mkdir -p gpurun_out/r5d
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u benchmarks/ffm_early_parity.py 500000 1 8 32 64 128 0 > gpurun_out/r5d/early_grid_curve.jsonl 2> gpurun_out/r5d/early.err
