#!/bin/bash
# Extra single-GPU measurements (GPU box via gpurun): the headline C2 line plus C3, C5 (SORTING) and
# the churn log (overwrites + DELETEs, exact segment replay).  Each run has its own time limit.
#   tools/workloads.sh TAG [entries for c3/c5]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-wl}
N3=${2:-100000000}
mkdir -p $OUT
echo churn && timeout -k 10 300 python -u bench.py --workload churn --steps 5 --warmup 1 > $OUT/churn.log 2>&1 &&
echo c3 && timeout -k 10 400 python -u bench.py --workload c3 --entries $N3 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/c3.log 2>&1 &&
echo c5 && timeout -k 10 400 python -u bench.py --workload c5 --entries $N3 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/c5.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
