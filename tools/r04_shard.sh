#!/bin/bash
# Sharded receive into fixed bucket regions (k_part2_recv) on gpurun: the sharded parity tests, then
# A/B of two library builds (ablib/$A.so, ablib/$B.so) on the sharded N = 1 build of 125M C2 records
# and on a gloo N = 8 rehearsal (eight ranks on this one GPU, 4M records each), then a kernel trace
# of the N = 1 sharded build with B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04shard}; A=${2:-shortw}; B=${3:-recv}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sharded_gpu.py tests/test_multi_gpu_abi.py -x -v --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for v in $A $B; do
  MASTER_ADDR=127.0.0.1 MASTER_PORT=29563 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 SPARKEY_GPU_LIB=$PWD/ablib/$v.so \
    timeout -k 10 300 python -u bench.py --sharded --entries 125000000 --steps 5 --warmup 1 --no-check \
    > $O/n1_$v.jsonl 2> $O/n1_$v.err || exit 1
  SPARKEY_GPU_LIB=$PWD/ablib/$v.so timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29564 bench.py --gpus 8 --backend gloo --entries 4000000 --steps 3 \
    --warmup 1 > $O/n8_$v.jsonl 2> $O/n8_$v.err || exit 1
done
MASTER_ADDR=127.0.0.1 MASTER_PORT=29565 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 SPARKEY_GPU_LIB=$PWD/ablib/$B.so \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_n1 -o run -- \
  python3 bench.py --sharded --entries 125000000 --steps 5 --warmup 1 --no-check > $O/trace_n1.log 2>&1 || exit 1
for f in $O/n1_*.jsonl $O/n8_*.jsonl; do
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], d['ms_per_step'], d.get('bit_identical_to_single_gpu'), {k: round(v, 3) for k, v in d['phase_ms_rank0'].items()})" $f
done
