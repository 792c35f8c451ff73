#!/bin/bash
# A/B of library builds on one box: tools/lib_ab.sh TAG ROUNDS WORKLOAD name=lib.so ... (a name's
# lib.so under sparkey-java_amd/lib/; "cur" = the working tree's libsparkey_gpu.so).  The runs
# alternate, ROUNDS times; stage times per run go to gpurun_out/TAG/ab.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; ROUNDS=$2; WL=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $ROUNDS); do
  for nl in "$@"; do
    name=${nl%%=*}; lib=$PWD/sparkey-java_amd/lib/${nl#*=}
    SPARKEY_GPU_LIB=$lib timeout -k 10 200 python -u bench.py --workload $WL --steps 10 --warmup 2 --no-cpu-baseline --quick > $OUT/${name}_$i.log 2>&1 || exit 1
    tail -1 $OUT/${name}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name $i', round(d['ms_per_step'],4), {k: round(v,4) for k, v in d['stage_ms'].items()})" >> $OUT/ab.txt
  done
done
echo done
