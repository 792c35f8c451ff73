#!/bin/bash
# C3 k_frame counters on the GPU box: kernel trace + SQ instruction / wait counters (separate passes).
#   tools/c3_prof.sh TAG [extra bench.py args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-c3prof}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS="--workload c3 --steps 2 --warmup 1 --no-cpu-baseline --quick $*"
echo "trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 &&
echo "sq" && timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1 &&
echo "sq2" && timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq2 -o run -- python3 bench.py $ARGS > $OUT/sq2.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
