#!/bin/bash
# Round-5 measurement pass (gpurun): the default bench line, the other workloads, rocprofv3 kernel
# stats of C2 and C3 100M, and their FETCH_SIZE / WRITE_SIZE passes (tools/pmc_summary.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05meas}; mkdir -p $O; P=profiles/r05_pmc_summary.json
b() { local n=$1; shift; timeout -k 10 600 python -u bench.py "$@" > $O/$n.jsonl 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }; tail -1 $O/$n.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step'],4), d.get('stage_ms'))"; }
b default && b c3_100m --workload c3 --entries 100000000 --steps 10 --warmup 2 --no-cpu-baseline \
  && b c5_100m --workload c5 --entries 100000000 --steps 10 --warmup 2 --no-cpu-baseline \
  && b c1x --workload c1x --steps 20 --warmup 3 --no-cpu-baseline && b churn --workload churn --steps 10 --warmup 2 --no-cpu-baseline \
  && b c4 --workload c4 --steps 3 --warmup 1 --no-cpu-baseline \
  && b snappy --workload snappy --steps 10 --warmup 2 --no-cpu-baseline && b zstd --workload zstd --steps 10 --warmup 2 --no-cpu-baseline || exit 1
for W in c2:"--workload c2" c3_100000000:"--workload c3 --entries 100000000"; do
  n=${W%%:*}; A="${W#*:} --steps 3 --warmup 1 --no-parity --no-cpu-baseline --quick"
  D=$O/rocprof_$n; mkdir -p $D
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $A > $D/trace.log 2>&1 || exit 1
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- python3 bench.py $A > $D/fetch.log 2>&1 || exit 1
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- python3 bench.py $A > $D/write.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $D $O/r05_pmc_summary.json $n > $D/summary.txt 2>&1 || exit 1
  head -20 $D/summary.txt
done
echo meas done
