#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05g5; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/pytest_parity.log 2>&1 || { tail -40 $O/pytest_parity.log; exit 1; }
tail -2 $O/pytest_parity.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_large.py -k "c3 or c5 or mixed or general" > $O/pytest_large.log 2>&1 || { tail -40 $O/pytest_large.log; exit 1; }
tail -2 $O/pytest_large.log
ABDEBUG=frame_debug ROUNDS=2 bash tools/r04_ab.sh r05g5/ab "--workload c3 --entries 10000000 --steps 5 --warmup 1" r04 new1 new2
ROUNDS=1 bash tools/r04_ab.sh r05g5/ab100 "--workload c3 --entries 100000000 --steps 5 --warmup 1" r04 new2
