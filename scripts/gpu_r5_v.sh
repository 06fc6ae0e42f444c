# round 5 v: every BASELINE config on one MI355X (fresh numbers for BASELINE.md)
set -o pipefail
mkdir -p gpurun_out/r5
for c in classifier linear_gpu linear_hashed fm gbdt rf bprmf xgboost; do
  timeout -k 10 300 python -u benchmarks/bench_configs.py $c >> gpurun_out/r5/bench_configs_r5.jsonl 2>> gpurun_out/r5/bench_configs_r5.err
  rc=$?; echo "$c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
