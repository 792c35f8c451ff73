#!/bin/bash
# k_frame3: base (committed) / v1 (the hash reads the chosen lists in place) / v2 (v1 + the entry
# search reads each head's list as four 64-bit words): framing tests on v2, C3 10M A/B, v2 phases.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab10}
mkdir -p $OUT
echo tests && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "frame3 or mixed or c3 or lane_matches or delete or random" > $OUT/tests.log 2>&1 &&
echo ab && bash tools/lib_ab.sh ${1:-ab10} 2 c3 base=libsparkey_gpu_base.so v1=libsparkey_gpu_v1.so v2=libsparkey_gpu.so > $OUT/lib_ab.log 2>&1 &&
echo phases && SPARKEY_FRAME_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --quick > $OUT/v2_phases.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
