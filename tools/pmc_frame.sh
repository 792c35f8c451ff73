#!/bin/bash
# SQ instruction counters of the bench kernels (one --pmc pass; no tracing domains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${1:-cur}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/log 2>&1
