#!/bin/bash
# Part B2: C5 at 100M, SNAPPY / ZSTD / churn benches, the host I/O probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-final_b2}
mkdir -p gpurun_out/$T
bash tools/final_r03.sh $T c5 comp io > gpurun_out/$T/steps.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
