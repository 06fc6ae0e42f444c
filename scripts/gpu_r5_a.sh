# round 5: FFM multi-hot deferral + hot-slot paths, fused delta mixing, FM adaptive bias refresh
set -o pipefail
mkdir -p gpurun_out/r5
ok() { case "$1" in 0|1) return 0;; *) echo "stop: rc=$1"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_ffm.py tests/test_mix_rccl.py tests/test_fm.py tests/test_linear.py tests/test_trees.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r5/pytest_a.log 2>&1
rc=$?; echo "pytest rc=$rc"; ok $rc
timeout -k 10 400 python -u benchmarks/ffm_hot_probe.py --hs 0,26,512,8192 --lds 27:16,27:32,27:8,8:16 > gpurun_out/r5/ffm_hot_probe.jsonl 2> gpurun_out/r5/ffm_hot_probe.err
rc=$?; echo "probe rc=$rc"; ok $rc
timeout -k 10 120 python -u benchmarks/mix_delta_probe.py > gpurun_out/r5/mix_delta_probe.jsonl 2> gpurun_out/r5/mix_delta_probe.err
rc=$?; echo "mix rc=$rc"; ok $rc
timeout -k 10 200 python -u benchmarks/bench_configs.py fm > gpurun_out/r5/bench_fm.jsonl 2> gpurun_out/r5/bench_fm.err
echo "fm rc=$?"
rc=0; ok $rc
HM_PROBE_MB=1024,8192 timeout -k 10 400 python -u benchmarks/linear_replica_probe.py 1000000 128 "-opt adam -eta0 0.01" "-opt sgd -eta0 0.05" "-opt rmsprop -eta0 0.01" "-opt adadelta" > gpurun_out/r5/linear_replica_probe.jsonl 2> gpurun_out/r5/linear_replica_probe.err
echo "linear rc=$?"
# same-box A/B: multi-hot detection on/off (hot path off), then the hot path on
for rep in 1 2; do
  for cfg in "HM_FFM_HOT=0 HM_FFM_DEFER=0" "HM_FFM_HOT=0 HM_FFM_DEFER=1" "HM_FFM_HOT=27 HM_FFM_DEFER=1"; do
    env $cfg timeout -k 10 150 python -u bench.py --steps 20 --warmup 8 --alt-run 0 > gpurun_out/r5/ab_bench.tmp 2>&1
    rc=$?; echo "$cfg rep $rep rc=$rc: $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*' gpurun_out/r5/ab_bench.tmp | tr '\n' ' ')" >> gpurun_out/r5/ab_bench.log
    ok $rc
  done
done
