# round 5 p: feature-lane histogram, prefetched gathers, branch-free staged adds -- tests, micro, GBDT, LDS counters
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
ok() { case "$1" in 0|1) return 0;; *) echo "stop: rc=$1"; exit "$1";; esac; }
timeout -k 10 400 python -u -m pytest tests/test_trees.py tests/test_xgboost.py -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r5/pytest_trees_p.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r5/pytest_trees_p.log; ok $rc
for fl in 0 1; do
  HM_HIST_FL=$fl timeout -k 10 200 python -u benchmarks/hist_micro.py > gpurun_out/r5/hist_micro4_fl$fl.jsonl 2>&1
  rc=$?; echo "micro fl=$fl rc=$rc"; ok $rc
done
for fl in 0 1 0 1; do
  echo "== fl $fl" >> gpurun_out/r5/gbdt_fl4_ab.log
  HM_HIST_FL=$fl timeout -k 10 300 python -u benchmarks/bench_configs.py gbdt >> gpurun_out/r5/gbdt_fl4_ab.log 2>&1
  rc=$?; echo "gbdt fl=$fl rc=$rc"; ok $rc
done
for fl in 0 1; do
  HM_HIST_FL=$fl timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r5/pmc_hist4_fl$fl -o run -- python3 benchmarks/hist_micro.py 4000000 > gpurun_out/r5/pmc_hist4_fl$fl.log 2>&1
  rc=$?; echo "pmc fl=$fl rc=$rc"; ok $rc
done
