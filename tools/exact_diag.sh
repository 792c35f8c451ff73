#!/bin/bash
# Exact path, one launch at a time (SPARKEY_EXACT_DEBUG=2): which kernel fails, segment counts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-xdiag}
mkdir -p $OUT
SPARKEY_EXACT_DEBUG=2 timeout -k 10 200 python -u bench.py --workload churn --entries ${2:-10000000} --steps 1 --warmup 0 --no-cpu-baseline > $OUT/diag.log 2>&1
rc=$?
grep -E "^\[exact|^\{|Error" $OUT/diag.log | cut -c1-300 | tail -30
exit $rc
