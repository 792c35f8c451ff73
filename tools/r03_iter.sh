#!/bin/bash
# One iteration: the full -m gpu suite, the C3 bench (10M), then the k_frame3 phase counters.
#   tools/r03_iter.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-it}
mkdir -p $OUT
echo pytest && timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
echo c3 && timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --quick > $OUT/c3.log 2>&1 &&
echo c2 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --quick > $OUT/c2.log 2>&1 &&
echo phases && bash tools/f3_phases.sh $1/f3ph > $OUT/f3ph.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
