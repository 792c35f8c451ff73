#!/bin/bash
# Sharded exact path on one GPU: the churn rehearsal at 1, 2, 4 ranks (threads of one
# process on cuda:0), then rocprofv3 kernel stats of the 2-rank rehearsal and of the single-GPU build
# (what the ranks' time is spent on: their kernels or each other's).   tools/r03_shard.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-shard}
mkdir -p $OUT
echo rehearsal && timeout -k 10 400 python -u tools/shard_rehearsal.py --entries 10000000 --ranks 1,2,4 --reps 2 > $OUT/rehearsal.log 2>&1 &&
echo prof2 && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof2 -o run -- python3 tools/shard_rehearsal.py --entries 10000000 --ranks 2 --reps 1 > $OUT/prof2.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
