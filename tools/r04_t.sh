#!/bin/bash
# Tests + C4 bench after partition changes (gpurun).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04t}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_c4.py tests/test_gpu_large.py tests/test_gpu_parity.py -x -v --timeout 600 \
  --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload c4 --steps 5 --warmup 1 > $O/bench_c4.jsonl 2> $O/bench_c4.err &&
timeout -k 10 300 python -u bench.py --workload c1x --steps 20 --warmup 3 > $O/c1x.jsonl 2> $O/c1x.err &&
SPARKEY_DEBUG=no_frame3=1 timeout -k 10 300 python -u bench.py --workload c1x --steps 20 --warmup 3 > $O/c1x_kframe.jsonl 2> $O/c1x_kframe.err
