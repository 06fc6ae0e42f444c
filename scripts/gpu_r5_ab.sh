# round 5 ab: train_fm grid vs parity spread, 5 reps of 128 / 160 / 192
set -o pipefail
mkdir -p gpurun_out/r5
export HM_NO_AUTOBUILD=1
PROBE_REPS=5 timeout -k 10 600 python -u benchmarks/fm_grid_parity_probe.py 128 160 192 > gpurun_out/r5/fm_grid_parity_ab.jsonl 2> gpurun_out/r5/fm_grid_parity_ab.err
rc=$?; echo "probe rc=$rc"; cat gpurun_out/r5/fm_grid_parity_ab.jsonl
