#!/bin/bash
# Partition changes on one GPU (gpurun): the placement/partition parity tests (C3 100M, the 20M k_part2f
# case, C2, churn), then the C3 100M and C2 bench lines and a rocprofv3 kernel summary of C3 100M.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04part}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py -x -v --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload c3 --entries 100000000 --steps 5 --warmup 1 > $O/c3_100m.jsonl 2> $O/c3_100m.err &&
SPARKEY_DEBUG=no_lookback=1 timeout -k 10 400 python -u bench.py --workload c3 --entries 100000000 --steps 5 --warmup 1 \
  > $O/c3_100m_nolb.jsonl 2> $O/c3_100m_nolb.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/c2.jsonl 2> $O/c2.err &&
SPARKEY_DEBUG=no_buckets=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-parity > $O/c2_nob.jsonl 2> $O/c2_nob.err &&
SPARKEY_DEBUG=no_buckets=1 timeout -k 10 400 python -u bench.py --workload c3 --entries 100000000 --steps 5 --warmup 1 \
  > $O/c3_100m_nob.jsonl 2> $O/c3_100m_nob.err &&
timeout -k 10 300 python -u bench.py --workload c1x --steps 20 --warmup 3 > $O/c1x.jsonl 2> $O/c1x.err &&
SPARKEY_DEBUG=no_frame3=1 timeout -k 10 300 python -u bench.py --workload c1x --steps 20 --warmup 3 --no-parity > $O/c1x_kframe.jsonl 2> $O/c1x_kframe.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3_100m -o run -- \
  python -u bench.py --workload c3 --entries 100000000 --steps 5 --warmup 1 --no-parity > $O/prof_c3_100m.log 2>&1
