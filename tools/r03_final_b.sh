#!/bin/bash
# Round-3 evidence, part B: C3 at 100M (cpu_baseline bit identity on the line) and its PMC passes
# keyed c3_100000000, C5 at 100M, SNAPPY / ZSTD / churn, the host I/O probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-final_b}
OUT=gpurun_out/$T
mkdir -p $OUT
bash tools/final_r03.sh $T ${STEPS:-c3 pmc3} > $OUT/steps.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
