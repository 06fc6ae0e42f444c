# round 5 c: is the FFM same-stream gap XCD-L2 coherence?  Same rows in flight on 8 XCDs vs one.
set -o pipefail
mkdir -p gpurun_out/r5
ok() { case "$1" in 0|1) return 0;; *) echo "stop: rc=$1"; exit "$1";; esac; }
PROBE_MEM=default,fine timeout -k 10 600 python -u benchmarks/ffm_xcd_probe.py 1048576 8 64 512 0 > gpurun_out/r5/ffm_xcd_probe.jsonl 2> gpurun_out/r5/ffm_xcd_probe.err
rc=$?; echo "xcd probe rc=$rc"; ok $rc
timeout -k 10 200 python -u -m pytest tests/test_fm.py tests/test_trees.py -m gpu -v --timeout 200 --timeout-method thread -k "parity or 5_to_8" > gpurun_out/r5/pytest_c.log 2>&1
echo "pytest rc=$?"
