# round 5 h: coherent re-read + write-through (variant 16) vs write-through alone (15) on the
# full grid: is the remaining gap the read-to-store window?
set -o pipefail
mkdir -p gpurun_out/r5
ok() { case "$1" in 0|1) return 0;; *) echo "stop: rc=$1"; exit "$1";; esac; }
PROBE_VARIANTS=16,10 PROBE_ONE_XCD=0 timeout -k 10 300 python -u benchmarks/ffm_xcd_probe.py 1048576 8 0 > gpurun_out/r5/ffm_reload_wt_probe.jsonl 2> gpurun_out/r5/ffm_reload_wt_probe.err
rc=$?; echo "probe rc=$rc"; ok $rc
