#!/bin/bash
# k_frame4 A/B on one GPU (gpurun): its parity tests, then the C3 bench (10M and 100M) with k_frame4 (two
# chunk sizes) and with k_frame3, per-wave phase counters, and a rocprofv3 kernel summary of 100M.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04f4}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_frame4.py -x -v --timeout 120 --timeout-method thread \
  > $O/pytest_f4.log 2>&1 &&
SPARKEY_DEBUG=frame4=1 timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 3 > $O/c3_f4.jsonl 2> $O/c3_f4.err &&
SPARKEY_DEBUG=frame4=1,frame4_c=128 timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 3 > $O/c3_f4_128.jsonl 2> $O/c3_f4_128.err &&
SPARKEY_DEBUG=frame4=0 timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 3 > $O/c3_f3.jsonl 2> $O/c3_f3.err &&
SPARKEY_DEBUG=frame4=1,frame_debug=1 timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 \
  > $O/c3_f4_dbg.jsonl 2> $O/c3_f4_dbg.err &&
SPARKEY_DEBUG=frame4=1,frame4_c=128,frame_debug=1 timeout -k 10 300 python -u bench.py --workload c3 --steps 1 --warmup 0 \
  > $O/c3_f4_128_dbg.jsonl 2> $O/c3_f4_128_dbg.err &&
SPARKEY_DEBUG=frame4=1 timeout -k 10 400 python -u bench.py --workload c3 --entries 100000000 --steps 5 --warmup 1 \
  > $O/c3_100m_f4.jsonl 2> $O/c3_100m_f4.err &&
SPARKEY_DEBUG=frame4=0 timeout -k 10 400 python -u bench.py --workload c3 --entries 100000000 --steps 5 --warmup 1 \
  > $O/c3_100m_f3.jsonl 2> $O/c3_100m_f3.err
