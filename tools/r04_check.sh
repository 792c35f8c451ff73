#!/bin/bash
# Round-4 GPU check (run on the GPU box through gpurun): smoke, then the GPU suite.  Each GPU step has
# its own time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 &&
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/$T/pytest_gpu.log 2>&1
