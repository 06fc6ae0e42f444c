# round 5 j: is the bench-stream gap concurrency at all?  One block (the sequential learner) on the
# bench's 12.6 M-row stream, and the full grid with 0 / 8 / 16 atomic ramp steps
set -o pipefail
mkdir -p gpurun_out/r5
ok() { case "$1" in 0|1) return 0;; *) echo "stop: rc=$1"; exit "$1";; esac; }
timeout -k 10 200 python -u benchmarks/ffm_hot_probe.py --hs "" --plain 0 --ramp-steps 0 >> gpurun_out/r5/ffm_stream_gap_src.jsonl 2>> gpurun_out/r5/ffm_stream_gap_src.err
rc=$?; echo "ramp0 rc=$rc"; ok $rc
timeout -k 10 200 python -u benchmarks/ffm_hot_probe.py --hs "" --plain 0 --ramp-steps 8 >> gpurun_out/r5/ffm_stream_gap_src.jsonl 2>> gpurun_out/r5/ffm_stream_gap_src.err
rc=$?; echo "ramp8 rc=$rc"; ok $rc
timeout -k 10 300 python -u benchmarks/ffm_hot_probe.py --hs "" --plain 0 --ramp-steps 24 >> gpurun_out/r5/ffm_stream_gap_src.jsonl 2>> gpurun_out/r5/ffm_stream_gap_src.err
rc=$?; echo "ramp24 rc=$rc"; ok $rc
timeout -k 10 400 python -u benchmarks/ffm_hot_probe.py --hs "" --plain 0 --ramp-steps 0 --grid 1 --warmup 0 >> gpurun_out/r5/ffm_stream_gap_src.jsonl 2>> gpurun_out/r5/ffm_stream_gap_src.err
rc=$?; echo "grid1 rc=$rc"; ok $rc
