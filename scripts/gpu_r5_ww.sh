# round 5 ww: linear records mixed as one [NF, 4] row view -- RCCL one-rank mix tests, 2- and 4-rank gloo rehearsal of bench.py
set -o pipefail
mkdir -p gpurun_out/r5
export HM_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_mix_rccl.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r5/pytest_mix_ww.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r5/pytest_mix_ww.log; [ $rc -eq 0 ] || exit $rc
for n in 2 4; do
  HM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 2953$n bench.py --gpus $n --steps 12 --warmup 3 > gpurun_out/r5/rehearsal_ww_$n.log 2>&1
  rc=$?; echo "ranks=$n rc=$rc $(grep -o '"value": [0-9.]*\|"logloss_heldout": [0-9.]*\|"mixes_timed": [0-9]*\|"logloss_heldout_bf16": [0-9.]*' gpurun_out/r5/rehearsal_ww_$n.log | tr '\n' ' ')"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r5/rehearsal_ww_$n.log; exit $rc; }
done
