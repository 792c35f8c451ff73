#!/bin/bash
# rocprofv3 passes on the C2 bench (run on the GPU box via gpurun).  Kernel trace + stats first, then
# one PMC pass per counter group (never combined with tracing domains).  Usage: tools/profile.sh [pmc]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="--steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit 1
if [ "$1" = "pmc" ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1 || exit 1
fi
echo "profile done"
