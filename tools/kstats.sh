#!/bin/bash
# Per-kernel stats of one bench workload for library variants (gpurun):
#   kstats.sh TAG "bench args" NAME ...   -> gpurun_out/TAG/NAME_kernel_stats.csv
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1; ARGS=$2; shift 2
O=gpurun_out/$T; mkdir -p $O
for v in "$@"; do
  SPARKEY_GPU_LIB=$PWD/ablib/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- \
    python3 -u bench.py $ARGS --no-parity --no-cpu-baseline > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  f=$(find $O/prof_$v -name '*kernel_stats.csv' | head -1)
  cp "$f" $O/${v}_kernel_stats.csv
  echo "== $v"; cut -d, -f1-4 $O/${v}_kernel_stats.csv | head -12
done
