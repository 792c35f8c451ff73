#!/bin/bash
# One GPU session: smoke, parity tests, short bench.  Each GPU step has its own time limit and the
# chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 10 --warmup 2 "$@" > gpurun_out/bench.log 2>&1
