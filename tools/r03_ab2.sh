#!/bin/bash
# k_part2s pipelined + k_place_reg default: parity subset, C2/C3 quick benches, k_part2s phases.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab2}
mkdir -p $OUT
Q="--steps 10 --warmup 2 --no-cpu-baseline --quick"
echo tests && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 &&
echo c2 && timeout -k 10 200 python -u bench.py $Q > $OUT/c2.log 2>&1 &&
echo c3 && timeout -k 10 200 python -u bench.py --workload c3 $Q > $OUT/c3.log 2>&1 &&
echo part2dbg && SPARKEY_PART2_DEBUG=1 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --quick > $OUT/part2_dbg.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
