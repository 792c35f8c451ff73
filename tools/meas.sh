#!/bin/bash
# Measurement pass (gpurun): the default bench line, the other workloads, rocprofv3 kernel stats of
# C2, C3 100M and C4 (1B) with their FETCH_SIZE / WRITE_SIZE passes (tools/pmc_summary.py into
# $O/pmc_summary.json), the sharded 125M-record rank at N = 1 (the weak-scaling point), and a 2-rank
# gloo rehearsal whose line carries the one-GPU build of the same log.
#   usage: tools/meas.sh TAG [parts]   parts: any of bench,prof,c4prof,shardprof,shard (default: all but shardprof)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-meas}; mkdir -p $O
PARTS=${2:-bench,prof,c4prof,shard}
has() { [[ ",$PARTS," == *",$1,"* ]]; }
( while sleep 50; do echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &  # (long passes print nothing)
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
b() { local n=$1; shift; timeout -k 10 600 python -u bench.py "$@" > $O/$n.jsonl 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }; tail -1 $O/$n.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step'],4), d.get('stage_ms'))"; }
if has bench; then
  b default && b c3_100m --workload c3 --entries 100000000 --steps 10 --warmup 2 --no-cpu-baseline \
    && b c5_100m --workload c5 --entries 100000000 --steps 10 --warmup 2 --no-cpu-baseline \
    && b c1x --workload c1x --steps 20 --warmup 3 --no-cpu-baseline && b churn --workload churn --steps 10 --warmup 2 --no-cpu-baseline \
    && b c4 --workload c4 --steps 3 --warmup 1 --no-cpu-baseline \
    && b snappy --workload snappy --steps 10 --warmup 2 --no-cpu-baseline && b zstd --workload zstd --steps 10 --warmup 2 --no-cpu-baseline || exit 1
fi
prof() {  # name "bench args"
  local n=$1 A="$2"
  D=$O/rocprof_$n; mkdir -p $D
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $A > $D/trace.log 2>&1 || return 1
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- python3 bench.py $A > $D/fetch.log 2>&1 || return 1
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- python3 bench.py $A > $D/write.log 2>&1 || return 1
  python3 tools/pmc_summary.py $D $O/pmc_summary.json $n > $D/summary.txt 2>&1 || return 1
  head -20 $D/summary.txt
}
if has prof; then
  prof c2 "--workload c2 --steps 3 --warmup 1 --no-parity --no-cpu-baseline --quick" || exit 1
  prof c3_100000000 "--workload c3 --entries 100000000 --steps 3 --warmup 1 --no-parity --no-cpu-baseline --quick" || exit 1
fi
if has c4prof; then  # 1B: the kernel trace; counters at 700M (the WRITE_SIZE pass at 1B hangs in the profiler)
  D=$O/rocprof_c4_1000000000; mkdir -p $D
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py \
    --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $D/trace.log 2>&1 || exit 1
  prof c4_700000000 "--workload c4 --entries 700000000 --steps 2 --warmup 1 --no-cpu-baseline" || exit 1
fi
if has shardprof; then  # a sharded rank's kernels and traffic (N = 1: no exchange, the rank's own steps)
  prof sharded_rank_125000000 "--sharded --entries 125000000 --steps 2 --warmup 1 --no-check" || exit 1
fi
if has shard; then
  timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29592 bench.py --sharded --entries 125000000 --steps 5 --warmup 1 \
    > $O/sharded_n1_125m.jsonl 2> $O/sharded_n1_125m.err || { tail -20 $O/sharded_n1_125m.err; exit 1; }
  tail -1 $O/sharded_n1_125m.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('sharded n1', d['ms_per_step'], d['bit_identical_to_single_gpu'], d['phase_ms_rank0'], d['one_gpu_same_log'])"
  timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29593 bench.py --gpus 2 --backend gloo --entries 50000000 --steps 2 --warmup 1 \
    > $O/gloo_n2_50m.jsonl 2> $O/gloo_n2_50m.err || { tail -20 $O/gloo_n2_50m.err; exit 1; }
  tail -1 $O/gloo_n2_50m.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gloo n2', d['ms_per_step'], d['bit_identical_to_single_gpu'], d['one_gpu_same_log'])"
fi
echo meas done
