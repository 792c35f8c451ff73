#!/bin/bash
# Round-4 partition choice check (gpurun): parity tests, then C2, C3 100M (bucket regions and digit
# regions), and C1x with k_frame3's per-wave debug.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04b}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py tests/test_gpu_compressed.py -x -v --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/c2.jsonl 2> $O/c2.err &&
timeout -k 10 400 python -u bench.py --workload c3 --entries 100000000 --steps 5 --warmup 1 > $O/c3_100m.jsonl 2> $O/c3_100m.err &&
SPARKEY_DEBUG=no_buckets=1 timeout -k 10 400 python -u bench.py --workload c3 --entries 100000000 --steps 5 --warmup 1 \
  --no-parity > $O/c3_100m_nob.jsonl 2> $O/c3_100m_nob.err
