#!/bin/bash
# persistent placement A/B (same box), C2 quick benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab4}
mkdir -p $OUT
Q="--steps 20 --warmup 3 --no-cpu-baseline --quick"
echo tests && timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "overwrite or equal or uniform or bucket" > $OUT/tests.log 2>&1 &&
echo c2a && timeout -k 10 200 python -u bench.py $Q > $OUT/c2_a.log 2>&1 &&
echo c2p && SPARKEY_PLACE_PERSIST=1 timeout -k 10 200 python -u bench.py $Q > $OUT/c2_p.log 2>&1 &&
echo c2b && timeout -k 10 200 python -u bench.py $Q > $OUT/c2_b.log 2>&1 &&
echo c2pp && SPARKEY_PLACE_PERSIST=1 timeout -k 10 200 python -u bench.py $Q > $OUT/c2_pp.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
