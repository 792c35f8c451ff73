#!/bin/bash
# LDS / issue counters for the placement and partition kernels (one rocprofv3 --pmc pass each, no
# tracing in the same run).  Run on the GPU box: bash tools/pmc_place.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmcp}
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/a -o run -- python3 bench.py $ARGS > $OUT/a.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAVES SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/b -o run -- python3 bench.py $ARGS > $OUT/b.log 2>&1
echo "done rc=$?"
