#!/bin/bash
# k_frame3 at 6 waves per SIMD (keys hashed out of LDS only): its parity tests, then the region sweep
# on C3 10M (8 KiB regions fit 4 workgroups per CU, 4-6 KiB ones more); then the N = 2 rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab8}
mkdir -p $OUT
echo tests && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "frame3 or mixed or c3 or lane_matches or delete" > $OUT/tests.log 2>&1 &&
echo sweep && bash tools/f3_sweep.sh ${1:-ab8}/f3s "X=0" "SPARKEY_FRAME_REGION=6144" "SPARKEY_FRAME_REGION=4096" "SPARKEY_FRAME_REGION=5120" "X=1" > $OUT/sweep.log 2>&1 &&
echo scale && bash tools/r03_scale.sh ${1:-ab8}/scale > $OUT/scale.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
