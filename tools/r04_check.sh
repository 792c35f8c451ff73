#!/bin/bash
# Round-4 end-of-round GPU check (gpurun): smoke, the whole GPU suite, the default bench line, and a
# rocprofv3 kernel trace + stats of the default bench.  Each GPU step has its own time limit and the
# chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread ${PYTEST_ARGS} \
  > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench_default.jsonl 2> $O/bench_default.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rocprof_default -o run -- \
  python3 bench.py --steps 20 --warmup 3 --no-parity --no-cpu-baseline > $O/rocprof_default.log 2>&1
