#!/bin/bash
# Sharded SNAPPY / ZSTD bench rehearsals on one GPU (gpurun): every rank on this GPU, collectives over
# gloo on host buffers, each line checked against rank 0's single-GPU build of the whole log.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-czrehearse}; mkdir -p $O
( while sleep 50; do echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &
HB=$!
rc=0
run() {  # name nproc entries workload port
  timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $2 --master-addr 127.0.0.1 \
    --master-port $5 bench.py --gpus $2 --backend gloo --workload $4 --entries $3 --steps 3 --warmup 1 \
    > $O/$1.jsonl 2> $O/$1.err || { tail -20 $O/$1.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'],3), d['bit_identical_to_single_gpu'], {k: round(v,3) for k,v in d['phase_ms_rank0'].items()})" $O/$1.jsonl
}
run snappy_n2 2 10000000 snappy 29581 && run zstd_n2 2 10000000 zstd 29582 && run snappy_n4 4 5000000 snappy 29583 || rc=1
kill $HB
exit $rc
