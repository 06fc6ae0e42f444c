# round 5 b: FFM reload-delta variant (10) vs default on the bench stream; FM bias re-read schedules;
# the failing GPU tests of run a; bench A/B default vs variant 10
set -o pipefail
mkdir -p gpurun_out/r5
ok() { case "$1" in 0|1) return 0;; *) echo "stop: rc=$1"; exit "$1";; esac; }
timeout -k 10 300 python -u benchmarks/ffm_hot_probe.py --hs "" --plain 0,10,0,10 > gpurun_out/r5/ffm_reload_delta.jsonl 2> gpurun_out/r5/ffm_reload_delta.err
rc=$?; echo "ffm probe rc=$rc"; ok $rc
timeout -k 10 300 python -u -m pytest tests/test_fm.py tests/test_trees.py -m gpu -v --timeout 200 --timeout-method thread -k "parity or 5_to_8" > gpurun_out/r5/pytest_b.log 2>&1
rc=$?; echo "pytest rc=$rc"; ok $rc
timeout -k 10 400 python -u benchmarks/fm_w0_probe.py 3145728 1:0:0 8:0:1048576 8:2:1048576 8:0.5:0 > gpurun_out/r5/fm_w0_probe.jsonl 2> gpurun_out/r5/fm_w0_probe.err
rc=$?; echo "fm probe rc=$rc"; ok $rc
timeout -k 10 200 python -u benchmarks/bench_configs.py fm > gpurun_out/r5/bench_fm_b.jsonl 2> gpurun_out/r5/bench_fm_b.err
echo "fm bench rc=$?"
