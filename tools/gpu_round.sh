#!/bin/bash
# One GPU session (run on the GPU box via gpurun): smoke, parity tests, bench, the k_frame phase
# breakdown, and optionally a rocprofv3 kernel trace + stats of the bench and the PMC passes (each its
# own run, never combined with tracing).  Every GPU step has its own time limit; the chain stops at
# the first failure.
#   tools/gpu_round.sh TAG [tests|bench|prof|all] [extra bench.py args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-cur}
MODE=${2:-all}
shift 2 2>/dev/null
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --quick $*"
run_tests() {
  echo "smoke" && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
  echo "pytest" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
}
run_bench() {
  echo "bench" && timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 "$@" > $OUT/bench.log 2>&1 &&
  echo "frame debug" && SPARKEY_FRAME_DEBUG=1 SPARKEY_FILE_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $OUT/frame_debug.log 2>&1
}
run_prof() {
  echo "trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 &&
  echo "pmc" &&
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 &&
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1 &&
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/prof/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1 &&
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $OUT/prof/sq2 -o run -- python3 bench.py $ARGS > $OUT/sq2.log 2>&1
}
case $MODE in
  tests) run_tests ;;
  bench) run_bench "$@" ;;
  prof) run_prof ;;
  quick) run_tests && run_bench "$@" ;;
  all) run_tests && run_bench "$@" && run_prof ;;
esac
rc=$?
echo "done rc=$rc"
exit $rc
