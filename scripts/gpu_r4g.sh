#!/bin/bash
# FM: w0 shard refresh interval A/B; the SQL device feature chain after the device name
# formatting and int32 offsets; a GBDT tree-build kernel profile.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4g
mkdir -p $O
export HM_NO_AUTOBUILD=1
for rep in 1 2; do
  for e in 1 8 32; do
    echo "== fm w0_every $e rep $rep" >> $O/fm_ab.log
    HM_FM_W0_EVERY=$e timeout -k 10 300 python -u benchmarks/bench_configs.py fm >> $O/fm_ab.log 2>&1
  done
done
timeout -k 10 600 python -u benchmarks/sql_ftvec_bench.py 1000000 cuda arrow > $O/sql_ftvec.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gbdt -o gbdt -- \
  python3 benchmarks/bench_configs.py gbdt > $O/prof_gbdt.log 2>&1
# all-features single-pass histogram (FG=32, 1024-thread blocks) A/B
for w in 0 1; do
  echo "== hist_wide $w" >> $O/gbdt_ab.log
  HM_HIST_WIDE=$w timeout -k 10 300 python -u benchmarks/bench_configs.py gbdt >> $O/gbdt_ab.log 2>&1
done
HM_HIST_WIDE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gbdt_wide -o gbdt -- \
  python3 benchmarks/bench_configs.py gbdt > $O/prof_gbdt_wide.log 2>&1
HM_HIST_WIDE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_trees.py > $O/pytest_trees_wide.log 2>&1
