#!/bin/bash
# churn without the exact path's second framing (slabs reused): exact-path parity tests, churn bench;
# then the k_frame3 knob sweep on C3 10M.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab7}
mkdir -p $OUT
echo tests && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread -k "churn or exact or delete or overwrite or segment or dup or equal" > $OUT/tests.log 2>&1 &&
echo churn && timeout -k 10 300 python -u bench.py --workload churn --steps 5 --warmup 1 --no-cpu-baseline --quick > $OUT/churn.log 2>&1 &&
echo sweep && bash tools/f3_sweep.sh ${1:-ab7}/f3s "X=0" "SPARKEY_FRAME3_SHORT=1" "SPARKEY_FRAME3_SHORT=3" "SPARKEY_FRAME3_COVER=1" "SPARKEY_FRAME3_C=512" "SPARKEY_FRAME3_C=2048" "SPARKEY_FRAME_REGION=16384" "SPARKEY_FRAME3_C=512 SPARKEY_FRAME_REGION=4096" "X=1" > $OUT/sweep.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
