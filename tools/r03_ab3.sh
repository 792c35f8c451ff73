#!/bin/bash
# Placement sweep + init kernel: parity, smoke, C2/C3 quick benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab3}
mkdir -p $OUT
Q="--steps 20 --warmup 3 --no-cpu-baseline --quick"
echo tests && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_sharded_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 &&
echo smoke && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
echo c2 && timeout -k 10 200 python -u bench.py $Q > $OUT/c2.log 2>&1 &&
echo c2old && SPARKEY_PLACE_LDS=1 SPARKEY_NO_P2_STAGED=1 timeout -k 10 200 python -u bench.py $Q > $OUT/c2_old.log 2>&1 &&
echo p2dbg && SPARKEY_PART2_DEBUG=1 timeout -k 10 200 python -u tools/p2_probe.py > $OUT/p2dbg.log 2>&1 &&
echo c3 && timeout -k 10 200 python -u bench.py --workload c3 $Q > $OUT/c3.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
