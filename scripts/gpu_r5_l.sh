# round 5 l: roofline of the fp32 block layout with the driver's fld/val rows (mode 7), the RF
# 8-class GPU/CPU seed sweep, and the default bench
set -o pipefail
mkdir -p gpurun_out/r5
ok() { case "$1" in 0|1) return 0;; *) echo "stop: rc=$1"; exit "$1";; esac; }
MODES=5,7 timeout -k 10 200 python -u benchmarks/ffm_mem_roofline.py > gpurun_out/r5/roofline_fv.jsonl 2> gpurun_out/r5/roofline_fv.err
rc=$?; echo "roofline rc=$rc"; ok $rc
timeout -k 10 400 python -u benchmarks/rf_multiclass_probe.py 8 4 32 > gpurun_out/r5/rf_multiclass_probe.jsonl 2> gpurun_out/r5/rf_multiclass_probe.err
rc=$?; echo "rf rc=$rc"; ok $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r5/bench_l.log 2>&1
rc=$?; echo "bench rc=$rc"; ok $rc
