#!/bin/bash
# parity of the rewritten k_frame3 phases, then an A/B against the round-4 library (C3 10M)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05g3; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/pytest_parity.log 2>&1 || { tail -40 $O/pytest_parity.log; exit 1; }
tail -3 $O/pytest_parity.log
ABDEBUG=frame_debug ROUNDS=2 bash tools/r04_ab.sh r05g3/ab "--workload c3 --entries 10000000 --steps 5 --warmup 1" r04 new1
