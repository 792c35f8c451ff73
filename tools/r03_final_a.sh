#!/bin/bash
# Round-3 evidence, part A: smoke, the whole -m gpu suite, the default bench line (C2: cpu_baseline,
# parity leg, general framing, file->file), then its rocprofv3 kernel stats and PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-final_a}
mkdir -p $OUT
echo smoke && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
echo pytest && timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
echo bench && timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 > $OUT/bench_c2.log 2>&1 &&
echo pmc2 && bash tools/final_r03.sh ${1:-final_a}/pmc pmc2 > $OUT/pmc2.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
