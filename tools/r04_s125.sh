#!/bin/bash
# Single-GPU C2 shape at 125M records against the sharded N = 1 rank at the same size (gpurun):
# kernel traces of both, to compare k_frame_uniform per record.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04s125}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/single -o run -- \
  python3 bench.py --entries 125000000 --steps 5 --warmup 1 --no-parity --no-cpu-baseline > $O/single.log 2>&1 &&
MASTER_ADDR=127.0.0.1 MASTER_PORT=29566 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 \
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sharded -o run -- \
  python3 bench.py --sharded --entries 125000000 --steps 5 --warmup 1 --no-check > $O/sharded.log 2>&1
