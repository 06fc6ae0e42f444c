#!/bin/bash
# Round 3: sg32 kernel with G loaded into registers (52.6 KB LDS, 3 blocks/CU) (A/B
# against hivemall_amd/_lib_ab/libhm_hip_base.so), FFM GPU tests, then the SQL statement end to end.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HM_NO_AUTOBUILD=1
TAG=r3r bash scripts/gpu_ffm_ab.sh
