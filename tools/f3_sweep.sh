#!/bin/bash
# k_frame3 geometry sweep on the C3 shape (10M): the frame stage time per region size / knob setting.
#   tools/f3_sweep.sh TAG "ENV=V ..." ["ENV=V ..." ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-f3s}
shift
mkdir -p $OUT
i=0
for cfg in "$@"; do
  i=$((i+1))
  echo "cfg $i: $cfg" | tee -a $OUT/sweep.txt
  env $cfg timeout -k 10 200 python -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --quick > $OUT/c$i.log 2>&1 || exit 1
  tail -1 $OUT/c$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(' ms/build', round(d['ms_per_step'],4), {k: round(v,4) for k, v in d['stage_ms'].items()})" | tee -a $OUT/sweep.txt
done
echo "done"
