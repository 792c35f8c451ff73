#!/bin/bash
# k_frame_uniform with NB buffers per wave (SPARKEY_FRAME_NB): parity under NB=4, then A/B on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab6}
mkdir -p $OUT
Q="--steps 20 --warmup 3 --no-cpu-baseline --quick"
echo tests && SPARKEY_FRAME_NB=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q --timeout 200 --timeout-method thread -k "uniform or fixed or c2" > $OUT/tests.log 2>&1 &&
echo tests3 && SPARKEY_FRAME_NB=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "uniform" > $OUT/tests3.log 2>&1 &&
echo base && timeout -k 10 200 python -u bench.py $Q > $OUT/base.log 2>&1 &&
echo nb3 && SPARKEY_FRAME_NB=3 timeout -k 10 200 python -u bench.py $Q > $OUT/nb3.log 2>&1 &&
echo nb4 && SPARKEY_FRAME_NB=4 timeout -k 10 200 python -u bench.py $Q > $OUT/nb4.log 2>&1 &&
echo base2 && timeout -k 10 200 python -u bench.py $Q > $OUT/base2.log 2>&1 &&
echo nb4b && SPARKEY_FRAME_NB=4 timeout -k 10 200 python -u bench.py $Q > $OUT/nb4b.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
