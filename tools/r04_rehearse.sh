#!/bin/bash
# N = 2, 4, 8 rehearsals of the sharded bench on one GPU (gpurun): every rank on this GPU, collectives
# over gloo on host buffers, each line checked against one single-GPU build of the whole log.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04rehearse}
O=gpurun_out/$T
mkdir -p $O
for n in 2 4 8; do
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29570 + n)) bench.py --gpus $n --backend gloo --entries 4000000 --steps 3 --warmup 1 \
    > $O/n$n.jsonl 2> $O/n$n.err || exit 1
done
