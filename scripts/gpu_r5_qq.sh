# round 5 qq: train_fm parity vs the 8-mapper average, w in the V record vs a separate array
set -o pipefail
mkdir -p gpurun_out/r5
for sep in 0 1; do
  HM_FM_W_RECORD=$((1-sep)) timeout -k 10 400 python -u benchmarks/fm_grid_parity_probe.py 256 128 > gpurun_out/r5/fm_wrec_parity_$sep.jsonl 2> gpurun_out/r5/fm_wrec_parity_$sep.err
  rc=$?; echo "separate=$sep rc=$rc"; cat gpurun_out/r5/fm_wrec_parity_$sep.jsonl; [ $rc -eq 0 ] || exit $rc
done
