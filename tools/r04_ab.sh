#!/bin/bash
# A/B of library builds in ablib/ (gpurun): bench lines per variant, interleaved, two rounds.
# usage: r04_ab.sh TAG "bench args" variant...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1; ARGS=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    echo "== $v round $r" >> $O/ab.txt
    SPARKEY_DEBUG=${ABDEBUG:-} SPARKEY_GPU_LIB=$PWD/ablib/$v.so timeout -k 10 300 python -u bench.py $ARGS --no-parity --no-cpu-baseline \
      > $O/${v}_$r.jsonl 2> $O/${v}_$r.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d.get('stage_ms'))" \
      $O/${v}_$r.jsonl $v >> $O/ab.txt || exit 1
    grep '^\[k_frame\]' $O/${v}_$r.err | tail -1 >> $O/ab.txt
  done
done
cat $O/ab.txt
