# round 5 g: device-scope (SC1) slot loads / write-through stores vs the cross-XCD gap of the fp32
# FFM kernel: 1 M-row probe at 8 blocks and the full grid, then the bench stream
set -o pipefail
mkdir -p gpurun_out/r5
ok() { case "$1" in 0|1) return 0;; *) echo "stop: rc=$1"; exit "$1";; esac; }
PROBE_VARIANTS=0,13,14,15 PROBE_ONE_XCD=0 timeout -k 10 300 python -u benchmarks/ffm_xcd_probe.py 1048576 8 0 > gpurun_out/r5/ffm_sc1_probe.jsonl 2> gpurun_out/r5/ffm_sc1_probe.err
rc=$?; echo "sc1 probe rc=$rc"; ok $rc
PROBE_MEM=uncached PROBE_ONE_XCD=0 timeout -k 10 200 python -u benchmarks/ffm_xcd_probe.py 1048576 8 > gpurun_out/r5/ffm_uncached_xcd8.jsonl 2> gpurun_out/r5/ffm_uncached_xcd8.err
rc=$?; echo "uncached rc=$rc"; ok $rc
timeout -k 10 300 python -u benchmarks/ffm_hot_probe.py --hs "" --plain 13,14,15 > gpurun_out/r5/ffm_sc1_bench_stream.jsonl 2> gpurun_out/r5/ffm_sc1_bench_stream.err
rc=$?; echo "bench stream rc=$rc"; ok $rc
