#!/bin/bash
# A/B on one box: uniform framing direct loads (SPARKEY_FRAME_DIRECT=2/4) and persistent placement,
# with the uniform-log parity tests under the direct framing first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab5}
mkdir -p $OUT
Q="--steps 20 --warmup 3 --no-cpu-baseline --quick"
echo tests && SPARKEY_FRAME_DIRECT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "uniform or fixed or overwrite or equal" > $OUT/tests.log 2>&1 &&
echo smoke && SPARKEY_FRAME_DIRECT=2 timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
echo base && timeout -k 10 200 python -u bench.py $Q > $OUT/base.log 2>&1 &&
echo d2 && SPARKEY_FRAME_DIRECT=2 timeout -k 10 200 python -u bench.py $Q > $OUT/d2.log 2>&1 &&
echo d4 && SPARKEY_FRAME_DIRECT=4 timeout -k 10 200 python -u bench.py $Q > $OUT/d4.log 2>&1 &&
echo persist && SPARKEY_PLACE_PERSIST=1 timeout -k 10 200 python -u bench.py $Q > $OUT/persist.log 2>&1 &&
echo base2 && timeout -k 10 200 python -u bench.py $Q > $OUT/base2.log 2>&1 &&
echo d2b && SPARKEY_FRAME_DIRECT=2 timeout -k 10 200 python -u bench.py $Q > $OUT/d2b.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
