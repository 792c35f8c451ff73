#!/bin/bash
# Round-3 evidence on the GPU box: the headline bench line (C2, parity leg, cpu_baseline, general
# framing, file->file with phases), its rocprofv3 kernel stats and PMC passes, C3/C5 at 100M (with PMC
# keyed c3_100000000 and the CPU baseline's bit identity on the C3 line), SNAPPY / ZSTD / churn, the
# host I/O probe.  Each step has its own time limit; the chain stops at the first failure.
#   tools/final_r03.sh TAG [steps...]   (steps: c2 pmc2 c3 pmc3 c5 comp io; default all)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-final}
shift
STEPS=${*:-"c2 pmc2 c3 pmc3 c5 comp io"}
mkdir -p $OUT
Q="--steps 5 --warmup 1 --no-cpu-baseline --quick"
pmc() {  # $1 = tag, rest = bench args
  local t=$1; shift
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$t/trace -o run -- python3 bench.py "$@" > $OUT/$t.trace.log 2>&1 &&
  timeout -s KILL 420 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$t/fetch -o run -- python3 bench.py "$@" > $OUT/$t.fetch.log 2>&1 &&
  timeout -s KILL 420 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$t/write -o run -- python3 bench.py "$@" > $OUT/$t.write.log 2>&1 &&
  timeout -s KILL 420 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/$t/sq -o run -- python3 bench.py "$@" > $OUT/$t.sq.log 2>&1
}
rc=0
for st in $STEPS; do
  [ $rc -eq 0 ] || break
  echo "step $st"
  case $st in
    c2) timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 > $OUT/bench_c2.log 2>&1 ;;
    pmc2) pmc c2 $Q ;;
    c3) timeout -k 10 900 python -u bench.py --workload c3 --entries 100000000 --steps 5 --warmup 1 > $OUT/bench_c3.log 2>&1 ;;
    pmc3) pmc c3_100000000 --workload c3 --entries 100000000 $Q ;;
    c5) timeout -k 10 600 python -u bench.py --workload c5 --entries 100000000 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.log 2>&1 ;;
    comp) timeout -k 10 300 python -u bench.py --workload snappy --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_snappy.log 2>&1 &&
          timeout -k 10 300 python -u bench.py --workload zstd --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_zstd.log 2>&1 &&
          timeout -k 10 300 python -u bench.py --workload churn --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_churn.log 2>&1 ;;
    io) gcc -O2 -pthread tools/io_probe.c -o /tmp/io_probe && { nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; df -T /tmp; timeout -k 10 300 /tmp/io_probe /tmp; } > $OUT/io_probe.txt 2>&1 ;;
  esac
  rc=$?
done
echo "done rc=$rc"
exit $rc
