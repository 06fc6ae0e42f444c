# round 5 ii: what costs the -w0 path (experiment bits: 1 plain loads, 2 no shard loads, 4 no atomics)
set -o pipefail
mkdir -p gpurun_out/r5
for dbg in 0 1 2 4 6; do
  HM_FFM_BIAS_DBG=$dbg timeout -k 10 200 python -u benchmarks/ffm_w0_rate_probe.py > gpurun_out/r5/ffm_w0_dbg_$dbg.jsonl 2>&1
  echo "dbg=$dbg rc=$? $(grep -- '-w0' gpurun_out/r5/ffm_w0_dbg_$dbg.jsonl | head -1)"
done
