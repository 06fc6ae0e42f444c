# round 5 x: is train_fm's Hogwild gap lost updates?  fp32 V, store kernel vs every update by atomics
set -o pipefail
mkdir -p gpurun_out/r5
PROBE_OPTS="-fp32" PROBE_REPS=2 timeout -k 10 300 python -u benchmarks/fm_grid_parity_probe.py 256 128 > gpurun_out/r5/fm_atomic_probe.jsonl 2> gpurun_out/r5/fm_atomic_probe.err
echo "store rc=$?"
HM_FM_VARIANT=2 PROBE_OPTS="-fp32" PROBE_REPS=2 timeout -k 10 300 python -u benchmarks/fm_grid_parity_probe.py 256 128 >> gpurun_out/r5/fm_atomic_probe.jsonl 2>> gpurun_out/r5/fm_atomic_probe.err
echo "atomic rc=$?"
