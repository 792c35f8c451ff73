#!/bin/bash
# round 5: the C4 tests (300M against the oracle; 1B single GPU == 8 sharded ranks, byte for byte)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05c4; mkdir -p $O
timeout -k 10 1100 python -u -m pytest -x -v --timeout 1000 --timeout-method thread tests/test_gpu_c4.py > $O/pytest_c4.log 2>&1 || { tail -30 $O/pytest_c4.log; exit 1; }
tail -4 $O/pytest_c4.log
