#!/bin/bash
# Round 3: fused FFM predict kernel test + bench, mix device cost next to FFM, same-stream
# parity run (CPU-generated rows), counters of the shipped per-slot FFM kernels.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_sql_fused.py -m gpu -x -v --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r3l_pytest_fused.log
timeout -k 10 200 python benchmarks/mix_overlap_probe.py --world 8 2>&1 | tee gpurun_out/r3l_mix_overlap_w8.log
timeout -k 10 200 python benchmarks/mix_overlap_probe.py --world 2 2>&1 | tee gpurun_out/r3l_mix_overlap_w2.log
timeout -k 10 200 python benchmarks/mix_overlap_probe.py --world 8 --state fp32 2>&1 | tee gpurun_out/r3l_mix_overlap_w8_fp32.log
timeout -k 10 300 python bench.py --gen-device cpu 2>&1 | tee gpurun_out/r3l_bench_cpugen.log
OUT=ffm_pmc_sg12 PAT=ffm_pipe_sg12 bash scripts/ffm_counters.sh > gpurun_out/r3l_pmc_sg12.log 2>&1
FP32=1 OUT=ffm_pmc_psg32 PAT=ffm_pipe_sg32 bash scripts/ffm_counters.sh > gpurun_out/r3l_pmc_psg32.log 2>&1
timeout -k 10 400 python benchmarks/sql_ffm_predict_bench.py --rows 100000 --fields 10 --device cuda --generic 0 2>&1 | tee gpurun_out/r3l_sql_ffm_predict_gpu.log
