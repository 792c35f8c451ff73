#!/bin/bash
# Round-3 evidence after k_frame3's one-wave launch: the large-log GPU tests, C3 at 100M (CPU baseline
# bit identity) with its rocprofv3 / PMC passes, C5, SNAPPY / ZSTD / churn, the C2 headline line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-final_c}
OUT=gpurun_out/$T
mkdir -p $OUT
echo large && timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py -x -v --timeout 600 --timeout-method thread > $OUT/large.log 2>&1 &&
echo steps && bash tools/final_r03.sh $T c3 pmc3 c5 comp c2 > $OUT/steps.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
