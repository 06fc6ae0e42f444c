# round 5 mm: same-box A/B, HEAD kernel library (6ee...) vs the working tree's (linear state read in D)
set -o pipefail
mkdir -p gpurun_out/r5
for v in new head new head new head; do
  if [ $v = head ]; then export HM_HIP_LIB=$PWD/hivemall_amd/_lib/libhm_hip_head.so HM_NO_AUTOBUILD=1; else unset HM_HIP_LIB; unset HM_NO_AUTOBUILD; fi
  timeout -k 10 200 python -u bench.py > gpurun_out/r5/bench_ab_$v.log 2>&1
  rc=$?; echo "$v rc=$rc $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*\|"value_bf16_state": [0-9.]*' gpurun_out/r5/bench_ab_$v.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
