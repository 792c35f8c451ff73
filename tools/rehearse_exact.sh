#!/bin/bash
# Sharded exact path on one GPU (gpurun): per-rank phases of the threaded rehearsal at N = 1, 2, 4 and
# the kernel trace of the same runs (each kernel's own duration, apart from the ranks' waiting).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-rehearse_exact}; mkdir -p $O
timeout -k 10 300 python -u tools/shard_rehearsal.py --entries 10000000 --ranks 1,2,4 --reps 3 > $O/rehearsal.log 2>&1 || { tail -20 $O/rehearsal.log; exit 1; }
tail -30 $O/rehearsal.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/shard_rehearsal.py --entries 10000000 --ranks 1,2,4 --reps 1 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
echo rehearse done
