#!/bin/bash
# k_frame_lane (ring) iteration: the lane parity tests, smoke, the C3 10M fix-pass statistics and the
# kernel stats of a C3 bench (and of Z = 64 slices).   tools/r03_lane.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-lane}
mkdir -p $OUT
echo tests && timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "lane or spec or c3 or mixed" > $OUT/tests.log 2>&1 &&
echo smoke && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
echo lanedbg && SPARKEY_LANE_DEBUG=1 timeout -k 10 300 python3 -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu-baseline --quick > $OUT/lane_dbg.log 2>&1 &&
echo prof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline --quick > $OUT/prof.log 2>&1 &&
echo z64 && SPARKEY_LANE_Z=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof64 -o run -- python3 bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline --quick > $OUT/prof64.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
