# round 5 final evidence: every BASELINE config re-measured, kernel stats of the headline bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HM_NO_AUTOBUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out/r5/final
timeout -k 10 900 python -u benchmarks/bench_configs.py > gpurun_out/r5/final/configs.jsonl 2> gpurun_out/r5/final/configs.err
rc=$?; echo "configs rc=$rc"; cat gpurun_out/r5/final/configs.jsonl | cut -c1-260; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/final/ks -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/r5/final/bench_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/r5/final/bench_prof.log | cut -c1-200
