#!/bin/bash
# k_frame3 instructions by phase (C3, 10M): SPARKEY_FRAME3_STOP=k ends each wave after phase k (the build
# then reruns with k_frame, so only k_frame3's own counters are read); 9 = the whole kernel.  Prints
# k_frame3's per-launch counters for each k.   tools/f3_phases.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-f3ph}
mkdir -p $OUT
for k in 0 1 2 3 4 5 9; do
  echo "stop $k"
  SPARKEY_FRAME3_STOP=$k timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH --output-format csv -d $OUT/s$k -o run -- python3 bench.py --workload c3 --steps 1 --warmup 0 --no-cpu-baseline --quick > $OUT/s$k.log 2>&1 || exit 1
  python3 tools/pmc_kernels.py $(find $OUT/s$k -name "*counter_collection.csv") --kernels=k_frame3 | tee -a $OUT/phases.txt
done
echo "done"
