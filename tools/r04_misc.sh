#!/bin/bash
# Round-4 extras (gpurun): PMC passes of one rank of the sharded build at C4's per-GPU size (125M
# records, N = 1 over RCCL) for bench.py's N > 1 traffic figure, and the host file I/O probe
# (buffered, mmap and O_DIRECT writes) for the file -> file bound.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04misc}
O=gpurun_out/$T
mkdir -p $O
gcc -O2 -pthread tools/io_probe.c -o /tmp/io_probe && timeout -k 10 300 /tmp/io_probe /tmp > $O/io_probe.txt 2>&1 &&
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 &&
SQ= bash tools/r04_pmc.sh $T/pmc "sharded_rank_125000000:--sharded --entries 125000000 --no-check" &&
SQ=1 bash tools/r04_pmc.sh $T/pmc_c2 "c2:"
