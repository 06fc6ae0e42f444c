# round 5 f: does invalidating cached lines (variants 11/12) or uncached table memory close the
# fp32 FFM bench-stream gap (cross-XCD L2 staleness)?
set -o pipefail
mkdir -p gpurun_out/r5
ok() { case "$1" in 0|1) return 0;; *) echo "stop: rc=$1"; exit "$1";; esac; }
for ie in 1 16; do
  HM_FFM_INV_EVERY=$ie timeout -k 10 240 python -u benchmarks/ffm_hot_probe.py --hs "" --plain 11,12 >> gpurun_out/r5/ffm_inv_probe.jsonl 2>> gpurun_out/r5/ffm_inv_probe.err
  rc=$?; echo "inv $ie rc=$rc"; ok $rc
done
HM_FFM_MEM=uncached timeout -k 10 240 python -u benchmarks/ffm_hot_probe.py --hs "" --plain 0 > gpurun_out/r5/ffm_uncached_probe.jsonl 2> gpurun_out/r5/ffm_uncached_probe.err
rc=$?; echo "uncached rc=$rc"; ok $rc
