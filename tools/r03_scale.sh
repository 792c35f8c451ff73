#!/bin/bash
# The N > 1 bench path rehearsed on one GPU: N = 2 ranks over gloo (both on cuda:0, Python
# orchestrator), checked against a single-GPU build; once with one build, once with repeated builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-scale}
mkdir -p $OUT
echo n2a && timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --orchestrator python --entries 3000000 --steps 1 --warmup 0 --check > $OUT/n2a.log 2>&1 &&
echo n2b && timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --backend gloo --orchestrator python --entries 3000000 --steps 5 --warmup 1 --check > $OUT/n2b.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
