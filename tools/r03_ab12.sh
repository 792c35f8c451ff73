#!/bin/bash
# k_frame3 launch shape: waves per workgroup (4 default, 8, 1) with the region ticket or by workgroup
# id (SPARKEY_FRAME3_NOTICKET), C3 10M; framing tests with the 8-wave / no-ticket launches first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab12}
mkdir -p $OUT
echo tests && SPARKEY_FRAME3_WG=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "frame3 or mixed or c3" > $OUT/tests_wg8.log 2>&1 &&
SPARKEY_FRAME3_NOTICKET=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "frame3 or mixed or c3" > $OUT/tests_noticket.log 2>&1 &&
echo ab && bash tools/ab_env.sh ${1:-ab12} "X=0" "SPARKEY_FRAME3_NOTICKET=1" "SPARKEY_FRAME3_WG=8" "SPARKEY_FRAME3_WG=8 SPARKEY_FRAME3_NOTICKET=1" "SPARKEY_FRAME3_WG=1 SPARKEY_FRAME3_NOTICKET=1" "X=1" -- --workload c3 --quick > $OUT/ab.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
