#!/bin/bash
# The driver's N = 8 geometry rehearsed on one GPU (gpurun): 8 ranks x the default 125M records (C4's
# 1B in ONE index), every rank on this GPU, collectives over gloo on host buffers through the C++
# orchestrator, checked against rank 0's single-GPU build of the whole 1B log.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-rehearse8}; mkdir -p $O
( while sleep 50; do echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &
HB=$!
rc=0
timeout -k 10 1000 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29591 bench.py --gpus 8 --backend gloo --steps 2 --warmup 1 > $O/n8_125m.jsonl 2> $O/n8_125m.err || rc=1
kill $HB
[ -s $O/n8_125m.jsonl ] && python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['config']['entries'], d['ms_per_step'], d['bit_identical_to_single_gpu'], d.get('device_used_gb_after_timed_builds'), d['phase_ms_rank0'], d['check_s'], d['gen_s'])" $O/n8_125m.jsonl
[ $rc = 0 ] || tail -30 $O/n8_125m.err
exit $rc
