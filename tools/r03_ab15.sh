#!/bin/bash
# The framing kernels' DELETE counts into 64 spread counters (one device-wide counter serialised an
# atomic per wave): the GPU suite, then churn (its frame stage) and C3 / C2 quick lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab15}
mkdir -p $OUT
echo tests && timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
echo churn && timeout -k 10 300 python -u bench.py --workload churn --steps 5 --warmup 1 --no-cpu-baseline > $OUT/churn.log 2>&1 &&
echo c3 && timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --quick > $OUT/c3.log 2>&1 &&
echo c2 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --quick > $OUT/c2.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
