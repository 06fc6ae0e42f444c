#!/bin/bash
# Same-stream Hogwild parity on the field:index:value data (sequential CPU engine 0.44501,
# profiles/r4/ffm_parity_bench_scale_ffmdata.log) at several grids and kernels; DP mixing
# study (bf16, G-sum, mix interval); the SQL device feature-hashing bench; an FM epoch profile;
# the fixed tests.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4e
mkdir -p $O
export HM_NO_AUTOBUILD=1
for g in 0 1024 256; do
  echo "== grid $g" >> $O/parity.log
  timeout -k 10 300 python -u bench.py --gen-device cpu --grid $g --mix-probe 0 >> $O/parity.log 2>&1
done
echo "== generic kernel (variant 1)" >> $O/parity.log
HM_FFM_VARIANT=1 timeout -k 10 300 python -u bench.py --gen-device cpu --mix-probe 0 >> $O/parity.log 2>&1
timeout -k 10 600 python -u benchmarks/dp_sim.py --worlds 8 --rules mean --lr-power 0.5 0.75 1.0 --state bf16 \
  > $O/dp_sim_bf16.jsonl 2>&1
timeout -k 10 600 python -u benchmarks/dp_sim.py --worlds 8 --rules mean --gsum 1 --lr-power 0.5 1.0 --state fp32 \
  > $O/dp_sim_fp32_gsum.jsonl 2>&1
timeout -k 10 600 python -u benchmarks/dp_sim.py --worlds 8 --rules mean --mix-every 5 20 --lr-power 0.5 0.75 --state fp32 \
  > $O/dp_sim_fp32_interval.jsonl 2>&1
timeout -k 10 600 python -u benchmarks/sql_ftvec_bench.py 1000000 cuda arrow > $O/sql_ftvec.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fm -o fm -- \
  python3 benchmarks/bench_configs.py fm > $O/prof_fm.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_ffm.py tests/test_linear.py tests/test_sql.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || true
tail -4 $O/pytest.log
timeout -k 10 900 python -u benchmarks/linear_rules_parity.py 1000000 > $O/linear_rules.jsonl 2>&1
