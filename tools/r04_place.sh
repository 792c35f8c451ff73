#!/bin/bash
# k_place_reg with the wave-uniform rank loop (gpurun): parity tests, then C2 and C3 100M bench lines
# and a kernel trace of C2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04place}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_multi_gpu_abi.py \
  tests/test_sharded_gpu.py -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/c2.jsonl 2> $O/c2.err &&
timeout -k 10 400 python -u bench.py --workload c3 --entries 100000000 --steps 5 --warmup 1 --no-parity > $O/c3_100m.jsonl 2> $O/c3_100m.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c2 -o run -- \
  python3 bench.py --steps 20 --warmup 3 --no-parity --no-cpu-baseline > $O/trace_c2.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o run -- \
  python3 bench.py --workload c3 --entries 100000000 --steps 5 --warmup 1 --no-parity --no-cpu-baseline > $O/trace_c3.log 2>&1
