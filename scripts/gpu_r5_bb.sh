# round 5 bb: RandomForest (-mtry, depth 12) on fixed-shape heap levels: RF A/B (rate, AUC)
set -o pipefail
mkdir -p gpurun_out/r5
rm -f gpurun_out/r5/rf_heap_ab.log
for h in 1 0 1 0; do
  echo "== heap $h" >> gpurun_out/r5/rf_heap_ab.log
  HM_TREE_HEAP=$h timeout -k 10 300 python -u benchmarks/bench_configs.py rf >> gpurun_out/r5/rf_heap_ab.log 2>&1
  rc=$?; echo "rf heap=$h rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for h in 1 0; do
  HM_TREE_HEAP=$h timeout -k 10 300 python -u -m pytest tests/test_trees.py -m gpu -v -s --timeout 200 --timeout-method thread -k "rf_gpu_quality" > gpurun_out/r5/pytest_rfq_heap$h.log 2>&1
  echo "rfq heap=$h rc=$?"
done
