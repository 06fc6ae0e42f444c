# round 5 i: rows in flight per CU vs rate and gap (variants 17-19), 1 M-row probe and bench stream
set -o pipefail
mkdir -p gpurun_out/r5
ok() { case "$1" in 0|1) return 0;; *) echo "stop: rc=$1"; exit "$1";; esac; }
PROBE_VARIANTS=0,17,18,19 PROBE_ONE_XCD=0 timeout -k 10 300 python -u benchmarks/ffm_xcd_probe.py 1048576 0 > gpurun_out/r5/ffm_inflight_probe.jsonl 2> gpurun_out/r5/ffm_inflight_probe.err
rc=$?; echo "probe rc=$rc"; ok $rc
timeout -k 10 300 python -u benchmarks/ffm_hot_probe.py --hs "" --plain 0,17,18,19 > gpurun_out/r5/ffm_inflight_bench_stream.jsonl 2> gpurun_out/r5/ffm_inflight_bench_stream.err
rc=$?; echo "bench stream rc=$rc"; ok $rc
