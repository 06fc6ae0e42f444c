#!/bin/bash
# FFM early-training regime: first 500 K rows at full concurrency vs on fewer blocks.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4w
mkdir -p $O
export HM_NO_AUTOBUILD=1
timeout -k 10 900 python -u benchmarks/ffm_early_parity.py 500000 0 256 512 1024 2048 > $O/ffm_early.jsonl 2>&1
