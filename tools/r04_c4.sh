#!/bin/bash
# C4-size checks on one GPU (gpurun): the multi-GPU C-ABI tests, the 300M / 1B tests, the single-GPU
# C4 bench line and a 2-rank gloo rehearsal of the C++ orchestrator.  Each GPU step has its own time
# limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04c4}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_multi_gpu_abi.py tests/test_gpu_c4.py -x -v --timeout 600 \
  --timeout-method thread > gpurun_out/$T/pytest_c4.log 2>&1 &&
timeout -k 10 600 python -u bench.py --workload c4 --steps 5 --warmup 1 > gpurun_out/$T/bench_c4.jsonl 2> gpurun_out/$T/bench_c4.err &&
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --backend gloo --entries 10000000 --steps 5 --warmup 1 \
  > gpurun_out/$T/bench_n2_gloo.jsonl 2> gpurun_out/$T/bench_n2_gloo.err
