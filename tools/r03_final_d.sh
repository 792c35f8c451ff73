#!/bin/bash
# End-of-round check on the committed tree: smoke(), the default bench line (as the driver runs it),
# and the N = 2 rehearsal (gloo, Python orchestrator) against a single-GPU build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-final_d}
mkdir -p $OUT
echo smoke && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
echo bench && timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1 &&
echo scale && bash tools/r03_scale.sh ${1:-final_d}/scale > $OUT/scale.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
