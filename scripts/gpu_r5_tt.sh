# round 5 tt: same-stream gap, linear records with one 16-B access (lpack) vs three 4-B accesses vs separate arrays
set -o pipefail
mkdir -p gpurun_out/r5
for cfg in "HM_FFM_LPACK=0" "HM_FFM_LIN_SEPARATE=1" "HM_FFM_LPACK=1" "HM_FFM_LPACK=0" "HM_FFM_LIN_SEPARATE=1"; do
  env $cfg timeout -k 10 300 python -u bench.py --gen-device cpu > gpurun_out/r5/bench_tt.log 2>&1
  rc=$?; echo "$cfg rc=$rc $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*\|"value_bf16_state": [0-9.]*\|"logloss_heldout_bf16": [0-9.]*' gpurun_out/r5/bench_tt.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
