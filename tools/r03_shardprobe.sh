#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-sprobe}
mkdir -p $OUT
echo probe && timeout -k 10 600 python -u tools/shard_probe.py 300000,3000000,6000000 > $OUT/probe.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
