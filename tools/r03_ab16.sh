#!/bin/bash
# k_frame2 (opt-in, SPARKEY_FRAME2) with the one-wave launch against the 4-wave ticket launch, C3 10M;
# the GPU suite first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab16}
mkdir -p $OUT
echo tests && timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
echo ab && bash tools/ab_env.sh ${1:-ab16} "SPARKEY_FRAME2=1 SPARKEY_FRAME_TICKET=1" "SPARKEY_FRAME2=1" "SPARKEY_FRAME2=1 SPARKEY_FRAME_TICKET=1" "SPARKEY_FRAME2=1" -- --workload c3 --quick > $OUT/ab.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
