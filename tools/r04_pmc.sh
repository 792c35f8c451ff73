#!/bin/bash
# Round-4 rocprofv3 passes (gpurun): for each workload a kernel trace + stats run, then one PMC pass
# each for FETCH_SIZE and WRITE_SIZE (never combined with tracing), summarised per workload into
# gpurun_out/$T/r04_pmc_summary.json (tools/pmc_summary.py; bench.py reads the committed copy).
#   bash tools/r04_pmc.sh TAG "c2:" "c3:" "c3_100000000:--workload c3 --entries 100000000" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04pmc}
shift
O=gpurun_out/$T
mkdir -p $O
for spec in "$@"; do
  W=${spec%%:*}
  A="${spec#*:} --steps 3 --warmup 1 --no-parity --no-cpu-baseline"
  D=$O/$W
  mkdir -p $D
  echo "== $W: $A"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $A \
    > $D/trace.log 2>&1 || exit 1
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- python3 bench.py $A \
    > $D/fetch.log 2>&1 || exit 1
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- python3 bench.py $A \
    > $D/write.log 2>&1 || exit 1
  if [ -n "$SQ" ]; then
    timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      GRBM_GUI_ACTIVE --output-format csv -d $D/sq -o run -- python3 bench.py $A > $D/sq.log 2>&1 || exit 1
  fi
  python3 tools/pmc_summary.py $D $O/r04_pmc_summary.json $W > $D/summary.txt 2>&1 || exit 1
  cat $D/summary.txt
done
echo "pmc done"
