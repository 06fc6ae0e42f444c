#!/bin/bash
# round 6: counters of the round-6 headline kernels (fp32 sg32 and bf16 sg12, KEEP default), of
# bpr_pf3 / mf (refresh of the round-3 numbers), and the multi-rank rehearsal (gloo, 2 ranks on
# one card) of bench.py with the pipelined mix and the N = 2 sequential reference
set -o pipefail
O=gpurun_out/r6i
mkdir -p $O
export TMPDIR=/tmp HM_NO_AUTOBUILD=1
G1="FETCH_SIZE"
G2="WRITE_SIZE"
G3="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
G4="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"
G5="TCC_HIT_sum TCC_MISS_sum"
G6="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
run_passes() {   # name, env, command...
  local name=$1; shift; local envs=$1; shift
  local i=0
  for grp in "$G1" "$G2" "$G3" "$G4" "$G5" "$G6"; do
    i=$((i+1))
    env $envs timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/$name/p$i -o run -- "$@" > $O/${name}_p$i.log 2>&1 || { echo "$name pass $i failed"; return 1; }
  done
}
run_passes sg32 "BF16=0" python3 benchmarks/ffm_prof_target.py || exit 1
run_passes sg12 "BF16=1" python3 benchmarks/ffm_prof_target.py || exit 2
python scripts/pmc_summary.py $O/sg32 sg32 > $O/sg32_summary.json || exit 3
python scripts/pmc_summary.py $O/sg12 sg12 > $O/sg12_summary.json || exit 3
run_passes bpr "X=1" python3 benchmarks/pmc_target.py bprmf || exit 4
python scripts/pmc_summary.py $O/bpr bpr_pf3 20000000 > $O/bpr_summary.json || exit 4
run_passes mf "X=1" python3 benchmarks/pmc_target.py mf || exit 5
python scripts/pmc_summary.py $O/mf mf_kernel 20000000 > $O/mf_summary.json || exit 5
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/ktrace -o run -- python3 benchmarks/ffm_prof_target.py > $O/ktrace.log 2>&1 || exit 6
HM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > $O/rehearsal_w2.log 2>&1 || exit 7
timeout -k 10 200 python benchmarks/ffm_variant_exact.py 0 10 > $O/keep2_exact.jsonl 2> $O/keep2_exact.err || exit 8
for rep in 1 2 3; do
  for v in 0 10; do
    HM_FFM_VARIANT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --alt-run 0 > $O/bench_fp32_v${v}_r$rep.log 2>&1 || exit 9
    HM_FFM_VARIANT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --alt-run 0 --state bf16 > $O/bench_bf16_v${v}_r$rep.log 2>&1 || exit 10
  done
done
echo ok
