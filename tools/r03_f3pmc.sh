#!/bin/bash
# k_frame3 (C3 10M) issue / wait / LDS counters, one rocprofv3 pass per counter group.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-f3pmc}
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "pass $i: $grp" | tee -a $OUT/pmc.txt
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --quick > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?" | tee -a $OUT/pmc.txt; tail -5 $OUT/p$i.log >> $OUT/pmc.txt; continue; }
  python3 tools/pmc_kernels.py $(find $OUT/p$i -name "*counter_collection.csv") --kernels=k_frame3,k_frame_uniform,k_place_reg | tee -a $OUT/pmc.txt
done
echo done
