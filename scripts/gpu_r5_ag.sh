# round 5 ag: experiment -- register-G sg32 variant (53.4 KB LDS, 3 blocks/CU) vs default, same box
set -o pipefail
mkdir -p gpurun_out/r5
export HM_NO_AUTOBUILD=1
for v in 9 0 9 0; do
  HM_FFM_VARIANT=$v timeout -k 10 200 python -u bench.py > gpurun_out/r5/bench_rg_$v.log 2>&1
  rc=$?; echo "variant=$v rc=$rc $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*' gpurun_out/r5/bench_rg_$v.log | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r5/bench_rg_$v.log; exit $rc; }
done
