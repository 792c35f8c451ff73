#!/bin/bash
# Round-2 evidence on the GPU box: the headline bench line (C2, cpu_baseline, general framing,
# file->file), its rocprofv3 kernel stats and PMC passes (each its own run), C3/C5 at 100M, the
# compressed and churn workloads, and the sharded churn rehearsal.  Each step has its own time limit;
# the chain stops at the first failure.   tools/final_r02.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
Q="--steps 5 --warmup 1 --no-cpu-baseline --quick"
pmc() {  # $1 = tag, rest = bench args
  local t=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$t/trace -o run -- python3 bench.py "$@" > $OUT/$t.trace.log 2>&1 &&
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$t/fetch -o run -- python3 bench.py "$@" > $OUT/$t.fetch.log 2>&1 &&
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$t/write -o run -- python3 bench.py "$@" > $OUT/$t.write.log 2>&1 &&
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/$t/sq -o run -- python3 bench.py "$@" > $OUT/$t.sq.log 2>&1
}
echo pmc-c2 && pmc c2 $Q &&
echo pmc-c3 && pmc c3 --workload c3 $Q &&
echo bench && timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > $OUT/bench_c2.log 2>&1 &&
echo c3 && timeout -k 10 400 python -u bench.py --workload c3 --entries 100000000 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_c3.log 2>&1 &&
echo c5 && timeout -k 10 400 python -u bench.py --workload c5 --entries 100000000 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.log 2>&1 &&
echo snappy && timeout -k 10 300 python -u bench.py --workload snappy --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_snappy.log 2>&1 &&
echo zstd && timeout -k 10 300 python -u bench.py --workload zstd --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_zstd.log 2>&1 &&
echo churn && timeout -k 10 300 python -u bench.py --workload churn --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_churn.log 2>&1 &&
echo shard-n1 && timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --sharded --steps 10 --warmup 2 --check > $OUT/bench_shard_n1.log 2>&1 &&
echo shard-churn-n1 && timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --sharded --workload churn --steps 5 --warmup 1 --check > $OUT/bench_shard_churn_n1.log 2>&1
rc=$?
echo "done rc=$rc"
exit $rc
