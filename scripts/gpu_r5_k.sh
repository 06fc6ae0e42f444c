# round 5 k: FFM GPU tests after the experiment cleanup (incl. the criteo_ffm pinned parity test),
# then the BPR / FM data-parallel quality sims and the headline kernel's counter passes
set -o pipefail
mkdir -p gpurun_out/r5
ok() { case "$1" in 0|1) return 0;; *) echo "stop: rc=$1"; exit "$1";; esac; }
timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r5/pytest_ffm_k.log 2>&1
rc=$?; echo "pytest rc=$rc"; ok $rc
bash scripts/gpu_r5_d.sh
