# round 5 af: GPU checkpoint round trip of the record layouts
set -o pipefail
mkdir -p gpurun_out/r5
export HM_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_elastic.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r5/pytest_elastic_af.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/r5/pytest_elastic_af.log
