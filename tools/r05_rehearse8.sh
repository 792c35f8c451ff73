#!/bin/bash
# Rehearsals of the driver's N > 1 bench on one GPU (gpurun), every rank on this GPU with its
# collectives over gloo on host buffers (the C++ orchestrator through sparkey_shard_comm_create_host),
# each line checked against rank 0's single-GPU build of the whole log:
#   N = 2 at the default 125M records a rank (C4's per-GPU share: one rank's footprint and phases), and
#   N = 8 at 50M a rank (eight ranks of 125M exceed one GPU's 288 GB; the driver gives each its own).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05rehearse; mkdir -p $O
( while sleep 50; do echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &
HB=$!
rc=0
timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29578 bench.py --gpus 2 --backend gloo --steps 2 --warmup 1 > $O/n2_125m.jsonl 2> $O/n2_125m.err || rc=1
[ $rc = 0 ] && { timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29579 bench.py --gpus 8 --backend gloo --entries 50000000 --steps 2 --warmup 1 > $O/n8_50m.jsonl 2> $O/n8_50m.err || rc=1; }
kill $HB
for f in $O/n2_125m.jsonl $O/n8_50m.jsonl; do [ -s $f ] && python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['bit_identical_to_single_gpu'], d.get('device_used_gb_after_timed_builds'), d['phase_ms_rank0'], d['check_s'])" $f; done
exit $rc
