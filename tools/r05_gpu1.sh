#!/bin/bash
# round 5, first GPU pass: k_frame3 geometry parity, then a C3 10M A/B over chunk sizes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05g1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "frame3" > $O/pytest_frame3.log 2>&1 || { tail -30 $O/pytest_frame3.log; exit 1; }
tail -3 $O/pytest_frame3.log
ROUNDS=2 bash tools/r04_env_ab.sh r05g1/ab "--workload c3 --entries 10000000 --steps 10 --warmup 2" "-" "frame3_c=2048" "frame3_c=4096" "frame3_c=8192" "frame3_c=8192,frame_region=16384" "frame3_c=16384,frame_region=16384"
