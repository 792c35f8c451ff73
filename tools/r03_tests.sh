#!/bin/bash
# Round-3 GPU session: smoke, the whole -m gpu suite, then the k_frame3 per-phase cycle counters on the
# C3 shape (SPARKEY_FRAME_DEBUG).  Each GPU step has its own time limit; the chain stops at the first
# failure.   tools/r03_tests.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03}
mkdir -p $OUT
echo smoke && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
echo pytest && timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
echo c3-phases && SPARKEY_FRAME_DEBUG=1 timeout -k 10 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --quick > $OUT/c3_phases.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
