#!/bin/bash
# k_part2s cost attribution: its phase cycles with each of its operations dropped in turn
# (SPARKEY_P2_EXP; timings only, the bytes are wrong on purpose).   tools/r03_p2exp.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-p2exp}
mkdir -p $OUT
export SPARKEY_PART2_DEBUG=1
echo e0 && timeout -k 10 200 python -u tools/p2_probe.py > $OUT/e0.log 2>&1 &&
echo e1 && SPARKEY_P2_EXP=1 timeout -k 10 200 python -u tools/p2_probe.py > $OUT/e1.log 2>&1 &&
echo e2 && SPARKEY_P2_EXP=2 timeout -k 10 200 python -u tools/p2_probe.py > $OUT/e2.log 2>&1 &&
echo e3 && SPARKEY_P2_EXP=3 timeout -k 10 200 python -u tools/p2_probe.py > $OUT/e3.log 2>&1 &&
unset SPARKEY_PART2_DEBUG &&
echo tests && timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
