# round 5 zz: train_fm default grid 192 -- FM GPU tests (default grid bounded at 3e-3), config-2 rate
set -o pipefail
mkdir -p gpurun_out/r5
export HM_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests/test_fm.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r5/pytest_fm_zz.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "mappers8|passed|failed" gpurun_out/r5/pytest_fm_zz.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u benchmarks/bench_configs.py fm > gpurun_out/r5/fm_zz.log 2>&1
rc=$?; echo "fm rc=$rc $(grep -o '"rows_per_s": [0-9.]*\|"heldout_logloss_after_2_epochs": [0-9.]*' gpurun_out/r5/fm_zz.log | tr '\n' ' ')"
