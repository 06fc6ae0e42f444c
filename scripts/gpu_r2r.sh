#!/bin/bash
# Round 2 call r: LDA E-step kernel (tests + bench), FFM parity test bound, smoke.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG="${TAG:-r2r}"
timeout -k 10 400 python -u -m pytest tests/test_topic_recommend.py tests/test_ffm.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || echo "pytest rc=$?" >> gpurun_out/pytest_$TAG.log
grep -q "Fatal\|core dumped\|Timeout" gpurun_out/pytest_$TAG.log && exit 3
timeout -k 10 500 python -u benchmarks/lda_bench.py > gpurun_out/lda_bench_$TAG.log 2>&1
echo done
