# round 5 e: XCD replicas of the fp32 FFM table (tests, then the bench-stream parity sweep)
set -o pipefail
mkdir -p gpurun_out/r5
ok() { case "$1" in 0|1) return 0;; *) echo "stop: rc=$1"; exit "$1";; esac; }
timeout -k 10 200 python -u -m pytest tests/test_ffm.py tests/test_trees.py -m gpu -v --timeout 120 --timeout-method thread -k "xcd or 5_to_8 or multihot" > gpurun_out/r5/pytest_e.log 2>&1
rc=$?; echo "pytest rc=$rc"; ok $rc
timeout -k 10 500 python -u benchmarks/ffm_xrep_probe.py 1:0:0 8:10:0.75 8:10:0.5 8:10:0 8:5:0.75 8:20:0.75 > gpurun_out/r5/ffm_xrep_probe.jsonl 2> gpurun_out/r5/ffm_xrep_probe.err
echo "xrep probe rc=$?"
