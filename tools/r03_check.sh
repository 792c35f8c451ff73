#!/bin/bash
# Round-3 check on the GPU box: smoke, the -m gpu suite, C2 and C3 (10M) quick benches.
#   tools/r03_check.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-chk}
mkdir -p $OUT
echo smoke && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
echo pytest && timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
echo c2 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --quick > $OUT/c2.log 2>&1 &&
echo c3 && timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --quick > $OUT/c3.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
