#!/bin/bash
# k_frame3 with one-wave workgroups by workgroup id (the default now): the GPU parity suite, then the
# region sweep on C3 10M (one-wave workgroups pack LDS per wave, so smaller regions fit more waves).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab13}
mkdir -p $OUT
echo tests && timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
echo ab && bash tools/ab_env.sh ${1:-ab13} "X=0" "SPARKEY_FRAME_REGION=6144" "SPARKEY_FRAME_REGION=5120" "SPARKEY_FRAME_REGION=12288" "SPARKEY_FRAME3_WG=4 SPARKEY_FRAME3_TICKET=1" "X=1" -- --workload c3 --quick > $OUT/ab.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
