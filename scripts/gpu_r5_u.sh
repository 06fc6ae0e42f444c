# round 5 u: linear mini-batch engine over two epochs (batch-counter reset)
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest tests/test_linear.py -m gpu -v -s --timeout 300 --timeout-method thread -k "minibatch" > gpurun_out/r5/pytest_linear_u.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5/pytest_linear_u.log
