# round 5 jj: train_ffm -w0 quality (sharded bias re-read every 8 / 16 / 1 rows, single address) vs sequential
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 500 python -u benchmarks/ffm_w0_quality_probe.py > gpurun_out/r5/ffm_w0_quality.jsonl 2> gpurun_out/r5/ffm_w0_quality.err
echo "rc=$?"
for e in 8 16; do
  HM_FFM_BIAS_EVERY=$e timeout -k 10 200 python -u benchmarks/ffm_w0_rate_probe.py > gpurun_out/r5/ffm_w0_rate_every$e.jsonl 2>&1
  echo "every=$e rc=$? $(grep -- '-w0' gpurun_out/r5/ffm_w0_rate_every$e.jsonl | tr '\n' ' ')"
done
