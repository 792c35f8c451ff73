#!/bin/bash
# A/B of build-time switches on the GPU box: one bench.py run per environment setting, stage times
# side by side.  tools/ab_env.sh TAG "ENV=1 ENV2=0" "ENV3=1" ... [-- extra bench.py args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
CONFIGS=(); EXTRA=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; EXTRA=("$@"); break; fi
  CONFIGS+=("$1"); shift
done
i=0
for c in "${CONFIGS[@]}"; do
  echo "== $c" | tee -a $OUT/ab.txt
  env $c timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline "${EXTRA[@]}" > $OUT/ab_$i.log 2>&1 || exit 1
  python -c "
import json,sys
d=json.loads(open('$OUT/ab_$i.log').read().strip().splitlines()[-1])
print('ms %.4f' % d['ms_per_step'], {k: round(v,4) for k,v in d['stage_ms'].items()}, 'file', d.get('file_to_file_keys_per_s'))
" | tee -a $OUT/ab.txt
  i=$((i+1))
done
