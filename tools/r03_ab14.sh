#!/bin/bash
# k_frame with one-wave workgroups by workgroup id (default now) against the 4-wave ticket launch
# (SPARKEY_FRAME_TICKET), on C3 10M framed by k_frame (SPARKEY_NO_FRAME3); the GPU suite first; then
# k_frame3's phases on the churn log (its frame stage is 2x C3's per byte).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab14}
mkdir -p $OUT
echo tests && timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
echo ab && bash tools/ab_env.sh ${1:-ab14} "SPARKEY_NO_FRAME3=1 SPARKEY_FRAME_TICKET=1" "SPARKEY_NO_FRAME3=1" "SPARKEY_NO_FRAME3=1 SPARKEY_FRAME_TICKET=1" "SPARKEY_NO_FRAME3=1" -- --workload c3 --quick > $OUT/ab.log 2>&1 &&
echo churn && SPARKEY_FRAME_DEBUG=1 timeout -k 10 300 python -u bench.py --workload churn --steps 2 --warmup 1 --no-cpu-baseline --quick > $OUT/churn_phases.log 2>&1 &&
SPARKEY_FRAME_DEBUG=1 SPARKEY_NO_UNIFORM=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --quick > $OUT/c2_general_phases.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
