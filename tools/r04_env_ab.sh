#!/bin/bash
# A/B of SPARKEY_DEBUG switch settings (gpurun): one bench line per setting, interleaved, ROUNDS rounds.
# usage: r04_env_ab.sh TAG "bench args" "switches A" "switches B" ...   ("-" = none)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1; ARGS=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
n=0
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for v in "$@"; do
    i=$((i+1)); sw=$v; [ "$sw" = "-" ] && sw=
    SPARKEY_DEBUG=$sw timeout -k 10 300 python -u bench.py $ARGS --no-parity --no-cpu-baseline \
      > $O/v${i}_$r.jsonl 2> $O/v${i}_$r.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],4), {k: round(v,4) for k,v in d.get('stage_ms').items()})" \
      $O/v${i}_$r.jsonl "[$v]" >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
