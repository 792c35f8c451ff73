#!/bin/bash
# SQ issue/wait counters of one kernel (gpurun): where its waves' cycles go.
# usage: sq.sh TAG KERNEL "bench args" [lib]   (lib: a build in ablib/, default the in-tree one)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1; K=$2; A="$3 --steps 2 --warmup 1 --quick --no-parity --no-cpu-baseline"; L=$4
O=gpurun_out/$T; mkdir -p $O
[ -n "$L" ] && export SPARKEY_GPU_LIB=$PWD/ablib/$L.so
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 bench.py $A > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS \
  SQ_INST_CYCLES_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 bench.py $A > $O/p2.log 2>&1 || exit 1
python3 tools/sq_summary.py $O "$K" | tee $O/sq.txt
