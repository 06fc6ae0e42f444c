# round 5 ad: train_ffm -w0 bias re-read interval 16 / 32 / 64: quality vs sequential and option rates
set -o pipefail
mkdir -p gpurun_out/r5
export HM_NO_AUTOBUILD=1
timeout -k 10 400 python -u benchmarks/ffm_w0_quality_probe.py 16 32 64 > gpurun_out/r5/ffm_w0_every_quality.jsonl 2>/dev/null
rc=$?; echo "quality rc=$rc"; cat gpurun_out/r5/ffm_w0_every_quality.jsonl; [ $rc -eq 0 ] || exit $rc
for e in 16 32 64; do
  HM_FFM_BIAS_EVERY=$e timeout -k 10 300 python -u benchmarks/ffm_option_rate_sweep.py > gpurun_out/r5/ffm_w0_every_rate_$e.jsonl 2>/dev/null
  rc=$?; echo "every=$e rc=$rc $(grep -- '-w0' gpurun_out/r5/ffm_w0_every_rate_$e.jsonl | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
