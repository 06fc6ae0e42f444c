#!/bin/bash
# round 6 validation after KEEP = 2 and the sg12 16-B landing-zone read: FFM GPU tests, smoke,
# 3 benches, sg12 LDS counters
set -o pipefail
O=gpurun_out/r6j
mkdir -p $O
export TMPDIR=/tmp HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests/test_ffm.py tests/test_mix_rccl.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_ffm.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_r$rep.log 2>&1 || exit 3
done
BF16=1 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sg12 -o run -- python3 benchmarks/ffm_prof_target.py > $O/pmc_sg12.log 2>&1 || exit 4
python scripts/pmc_summary.py $O/pmc_sg12 sg12 > $O/sg12_lds_summary.json || exit 5
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sg32 -o run -- python3 benchmarks/ffm_prof_target.py > $O/pmc_sg32.log 2>&1 || exit 6
python scripts/pmc_summary.py $O/pmc_sg32 sg32 > $O/sg32_lds_summary.json || exit 7
echo ok
