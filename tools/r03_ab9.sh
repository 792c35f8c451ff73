#!/bin/bash
# k_frame3 A/B on one box: the committed kernel (lib/libsparkey_gpu_base.so) against the working tree's
# (lib/libsparkey_gpu.so), C3 10M, alternating; then per-phase cycles of both; N = 2 rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab9}
mkdir -p $OUT
BASE=$PWD/sparkey-java_amd/lib/libsparkey_gpu_base.so
echo tests && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "frame3 or mixed or c3 or lane_matches or delete or random" > $OUT/tests.log 2>&1 &&
for i in 1 2; do
  echo "ab $i" &&
  SPARKEY_GPU_LIB=$BASE timeout -k 10 200 python -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --quick > $OUT/base_$i.log 2>&1 &&
  timeout -k 10 200 python -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --quick > $OUT/new_$i.log 2>&1 || exit 1
done &&
echo phases && SPARKEY_GPU_LIB=$BASE SPARKEY_FRAME_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --quick > $OUT/base_phases.log 2>&1 &&
SPARKEY_FRAME_DEBUG=1 timeout -k 10 200 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --quick > $OUT/new_phases.log 2>&1 &&
echo scale && bash tools/r03_scale.sh ${1:-ab9}/scale > $OUT/scale.log 2>&1
rc=$?
for f in $OUT/base_?.log $OUT/new_?.log; do
  tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],4), {k: round(v,4) for k, v in d['stage_ms'].items()})" >> $OUT/ab.txt 2>/dev/null
done
echo "done rc=$rc"
exit $rc
