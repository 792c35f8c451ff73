#!/bin/bash
# A/B of library builds (ablib/NAME.so) and switch settings (gpurun): one bench line per variant,
# interleaved, ROUNDS rounds.  usage: ab.sh TAG "bench args" NAME[:switches] ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1; ARGS=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for v in "$@"; do
    i=$((i+1)); lib=${v%%:*}; sw=""; [ "$lib" != "$v" ] && sw=${v#*:}
    [ -n "$ABDEBUG" ] && sw="${sw:+$sw,}$ABDEBUG"
    SPARKEY_DEBUG=$sw SPARKEY_GPU_LIB=$PWD/ablib/$lib.so timeout -k 10 300 python -u bench.py $ARGS --no-parity --no-cpu-baseline \
      > $O/v${i}_$r.jsonl 2> $O/v${i}_$r.err || { tail -5 $O/v${i}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],4), {k: round(v,4) for k,v in d.get('stage_ms').items()})" \
      $O/v${i}_$r.jsonl "[$v]" >> $O/ab.txt || exit 1
    grep '^\[k_frame\]' $O/v${i}_$r.err | tail -1 >> $O/ab.txt
  done
done
cat $O/ab.txt
