#!/bin/bash
# Exact-path phase breakdown on the churn workload (GPU box via gpurun).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-xd}
mkdir -p $OUT
SPARKEY_EXACT_DEBUG=1 timeout -k 10 300 python -u bench.py --workload churn --steps 2 --warmup 0 --no-cpu-baseline > $OUT/xd.log 2>&1
rc=$?
grep -E "^\[exact|^\{" $OUT/xd.log | tail -4
exit $rc
