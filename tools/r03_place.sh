#!/bin/bash
# k_place_lds phase cycles (SPARKEY_PLACE_DEBUG) on C2, then the default bench line (file->file phases).
#   tools/r03_place.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-place}
mkdir -p $OUT
echo place-debug && SPARKEY_PLACE_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --quick > $OUT/place_dbg.log 2>&1 &&
echo bench && timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 > $OUT/bench_c2.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
