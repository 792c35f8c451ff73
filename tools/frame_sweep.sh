#!/bin/bash
# A/B sweep of k_frame geometries on the C2 bench (GPU box via gpurun).  Each variant is one short
# bench.py run under its own time limit; prints build ms and per-stage ms, and with DEBUG=1 the
# k_frame phase cycles.   Usage: tools/frame_sweep.sh TAG "ENV1" "ENV2" ...   (ENV "alt" = lib/alt)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-sweep}
shift
mkdir -p $OUT
i=0
for v in "$@"; do
  i=$((i + 1))
  envs=""
  if [ "$v" = "alt" ]; then envs="SPARKEY_GPU_LIB=$PWD/sparkey-java_amd/lib/alt/libsparkey_gpu.so"; else envs="$v"; fi
  echo "== $v" >> $OUT/sweep.txt
  env $envs timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline $BENCH_ARGS > $OUT/b$i.log 2>&1 || { echo "FAILED $v" >> $OUT/sweep.txt; exit 1; }
  python - $OUT/b$i.log >> $OUT/sweep.txt <<'EOF'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print("  ms %.3f  " % d["ms_per_step"] + " ".join("%s=%.3f" % kv for kv in d["stage_ms"].items()))
EOF
  if [ -n "$DEBUG" ]; then
    env $envs SPARKEY_FRAME_DEBUG=1 timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline 2>&1 | grep "k_frame" | tail -1 >> $OUT/sweep.txt || exit 1
  fi
done
cat $OUT/sweep.txt
