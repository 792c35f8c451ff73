#!/bin/bash
# Quick C2 check on the GPU box: the parity tests that cover the canonical path, then the C2 bench
# (quick: timed builds and stage times only) with optional env.  tools/quick_c2.sh TAG [tests]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-q}
mkdir -p $OUT
if [ "$2" = "tests" ]; then
  echo tests && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_sharded_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
fi
echo bench && timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --quick --no-cpu-baseline > $OUT/bench.log 2>&1 || exit 1
tail -n 1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms', d['ms_per_step'], 'stages', d['stage_ms'])"
