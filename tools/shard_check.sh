#!/bin/bash
# Sharded build on the GPU box.  MODE: tests (sharded GPU tests), n1 (the N=1 sharded bench over
# RCCL), n2 (a 2-rank gloo rehearsal, both ranks on cuda:0), n4 (4 ranks x 10M C2 records with
# gloo on cuda:0, checked against one single-GPU build), churn (the exact path: single GPU, sharded N=1
# over RCCL, a 4-rank gloo rehearsal, the last two checked against a single-GPU build), all.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-shard}
MODE=${2:-all}
mkdir -p $OUT
t() { echo tests && timeout -k 10 400 python -u -m pytest tests/test_sharded_gpu.py tests/test_gpu_large.py -x -v --timeout 300 -k "sharded" > $OUT/tests.log 2>&1; }
n1() { echo n1 && timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --sharded --steps 10 --warmup 2 > $OUT/n1.log 2>&1; }
n2() { echo n2 && timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --entries 3000000 --steps 5 --warmup 1 > $OUT/n2.log 2>&1; }
n4() { echo n4 && timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 4 --backend gloo --steps 3 --warmup 1 --check > $OUT/n4.log 2>&1; }
prof1() { echo prof1 && RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --sharded --steps 10 --warmup 2 > $OUT/prof1.log 2>&1; }
churn() { echo churn && timeout -k 10 300 python -u bench.py --workload churn --steps 5 --warmup 1 --quick --no-cpu-baseline > $OUT/churn_single.log 2>&1 &&
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29537 bench.py --sharded --workload churn --steps 5 --warmup 1 --check > $OUT/churn_n1.log 2>&1 &&
  timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29539 bench.py --gpus 4 --backend gloo --workload churn --entries 2500000 --steps 2 --warmup 1 --check > $OUT/churn_n4.log 2>&1; }
single() { echo single && timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --quick --no-cpu-baseline > $OUT/single.log 2>&1; }
case $MODE in
  prof1) prof1 ;;
  churn) churn ;;
  cmp) single && n1 ;;
  tests) t ;;
  n1) n1 ;;
  n2) n2 ;;
  n4) n4 ;;
  all) t && n1 && n2 ;;
esac
rc=$?
echo "done rc=$rc"
exit $rc
