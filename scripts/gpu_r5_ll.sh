# round 5 ll: linear-state DMA issued early with forwarding (HM_FFM_LIN_DEFER=2) -- FFM tests under it, A/B vs 1
set -o pipefail
mkdir -p gpurun_out/r5
HM_FFM_LIN_DEFER=2 timeout -k 10 400 python -u -m pytest tests/test_ffm.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r5/pytest_ffm_ll.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/r5/pytest_ffm_ll.log; [ $rc -eq 0 ] || exit $rc
for d in 2 1 2 1 2 1; do
  HM_FFM_LIN_DEFER=$d timeout -k 10 200 python -u bench.py > gpurun_out/r5/bench_lin2_$d.log 2>&1
  rc=$?; echo "lin_defer=$d rc=$rc $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*' gpurun_out/r5/bench_lin2_$d.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
