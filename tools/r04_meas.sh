#!/bin/bash
# Round-4 bench lines for the README / DESIGN tables (gpurun): C4's size on one GPU, SNAPPY, ZSTD,
# churn (exact path), C5 (SORTING, 10M).  Each step has its own time limit; the chain stops at the
# first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r04meas}
O=gpurun_out/$T
mkdir -p $O
for w in snappy zstd churn c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 2 > $O/$w.jsonl 2> $O/$w.err || exit 1
done
timeout -k 10 600 python -u bench.py --workload c4 --steps 5 --warmup 1 > $O/c4.jsonl 2> $O/c4.err
