#!/bin/bash
# Kernel-level evidence: rocprofv3 kernel stats of C3 10M with k_frame_lane and with k_frame3
# (SPARKEY_NO_LANE), the lane fix-pass statistics (SPARKEY_LANE_DEBUG), k_place_lds phase cycles on C2
# (SPARKEY_PLACE_DEBUG), then the default C2 bench line (file->file phases).
#   tools/r03_prof.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
Q="--workload c3 --steps 5 --warmup 1 --no-cpu-baseline --quick"
echo lane && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lane -o run -- python3 bench.py $Q > $OUT/lane.log 2>&1 &&
echo f3 && SPARKEY_NO_LANE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/f3 -o run -- python3 bench.py $Q > $OUT/f3.log 2>&1 &&
echo lanedbg && SPARKEY_LANE_DEBUG=1 timeout -k 10 300 python3 -u bench.py --workload c3 --steps 1 --warmup 0 --no-cpu-baseline --quick > $OUT/lane_dbg.log 2>&1 &&
echo place-debug && SPARKEY_PLACE_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --quick > $OUT/place_dbg.log 2>&1 &&
echo bench && timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 > $OUT/bench_c2.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
