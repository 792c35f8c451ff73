#!/bin/bash
# A/B of build knobs on C2 / C3 quick benches (stage times).  tools/r03_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
Q="--steps 10 --warmup 2 --no-cpu-baseline --quick"
echo tests && timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "lane or spec or c3 or mixed or place or bucket" > $OUT/tests.log 2>&1 &&
echo c2 && timeout -k 10 200 python -u bench.py $Q > $OUT/c2_default.log 2>&1 &&
echo c2reg && SPARKEY_PLACE_REG=1 timeout -k 10 200 python -u bench.py $Q > $OUT/c2_reg.log 2>&1 &&
echo c2regnt && SPARKEY_PLACE_REG=1 SPARKEY_PLACE_NT=1 timeout -k 10 200 python -u bench.py $Q > $OUT/c2_regnt.log 2>&1 &&
echo c3 && timeout -k 10 200 python -u bench.py --workload c3 $Q > $OUT/c3_default.log 2>&1 &&
echo c3reg && SPARKEY_PLACE_REG=1 timeout -k 10 200 python -u bench.py --workload c3 $Q > $OUT/c3_reg.log 2>&1 &&
echo part2dbg && SPARKEY_PART2_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --quick > $OUT/part2_dbg.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
