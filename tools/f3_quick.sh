#!/bin/bash
# k_frame3 iteration: the framing parity tests, then the C3 bench (10M) with per-phase cycles and its
# stage times.   tools/f3_quick.sh TAG [extra bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-f3q}
shift
mkdir -p $OUT
echo tests && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 &&
echo c3 && timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --quick "$@" > $OUT/c3.log 2>&1 &&
echo c3-phases && SPARKEY_FRAME_DEBUG=1 timeout -k 10 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --quick "$@" > $OUT/c3_phases.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
