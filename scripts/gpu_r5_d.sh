# round 5 d: DP quality of BPR / FM at N = 2/4/8 on one card; headline kernel counters
set -o pipefail
mkdir -p gpurun_out/r5
ok() { case "$1" in 0|1) return 0;; *) echo "stop: rc=$1"; exit "$1";; esac; }
timeout -k 10 500 python -u benchmarks/dp_sim_mf_fm.py --worlds 2 4 8 --powers 0 0.5 0.75 --what bpr > gpurun_out/r5/dp_sim_bpr.jsonl 2> gpurun_out/r5/dp_sim_bpr.err
rc=$?; echo "bpr rc=$rc"; ok $rc
timeout -k 10 500 python -u benchmarks/dp_sim_mf_fm.py --worlds 2 4 8 --powers 0 0.5 0.75 --what fm > gpurun_out/r5/dp_sim_fm.jsonl 2> gpurun_out/r5/dp_sim_fm.err
rc=$?; echo "fm rc=$rc"; ok $rc
MODES="0" timeout -k 10 600 bash scripts/gpu_r5_pmc.sh > gpurun_out/r5/pmc_run.log 2>&1
echo "pmc rc=$?"
