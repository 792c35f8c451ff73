#!/bin/bash
# Part B1: the large-log GPU tests (100M C3/C5 vs the oracle: k_part2d's first run), then C3 at 100M
# (cpu_baseline bit identity) and its rocprofv3 / PMC passes keyed c3_100000000.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-final_b1}
OUT=gpurun_out/$T
mkdir -p $OUT
echo large && timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py -x -v --timeout 600 --timeout-method thread > $OUT/large.log 2>&1 &&
echo c3 && bash tools/final_r03.sh $T c3 pmc3 > $OUT/steps.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
