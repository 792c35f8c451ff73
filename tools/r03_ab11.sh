#!/bin/bash
# k_frame3 with one-wave workgroups (default now) against 2 / 4 waves per workgroup, C3 10M; the
# framing tests first; then the residency counters of the one-wave launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab11}
mkdir -p $OUT
echo tests && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "frame3 or mixed or c3 or lane_matches or delete or random" > $OUT/tests.log 2>&1 &&
echo ab && bash tools/ab_env.sh ${1:-ab11} "SPARKEY_FRAME3_WG=4" "SPARKEY_FRAME3_WG=1" "SPARKEY_FRAME3_WG=2" "SPARKEY_FRAME_REGION=6144" "SPARKEY_FRAME3_WG=4" "X=1" -- --workload c3 --quick > $OUT/ab.log 2>&1 &&
echo pmc && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- python3 bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --quick > $OUT/p1.log 2>&1 &&
python3 tools/pmc_kernels.py $(find $OUT/p1 -name "*counter_collection.csv") --kernels=k_frame3 > $OUT/pmc.txt
rc=$?
echo "done rc=$rc"
exit $rc
