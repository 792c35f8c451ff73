#!/bin/bash
# k_place_reg's branch-free write-out for 8-, 12- and 16-byte slots (gpurun): parity tests, then the
# c1x (12-byte slots), C3 10M (8-byte) and C2 (16-byte) bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04slots}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_sharded_gpu.py \
  tests/test_multi_gpu_abi.py -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c1x --steps 20 --warmup 3 > $O/c1x.jsonl 2> $O/c1x.err &&
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline > $O/c3.jsonl 2> $O/c3.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/c2.jsonl 2> $O/c2.err
