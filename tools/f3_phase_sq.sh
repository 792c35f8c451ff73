#!/bin/bash
# k_frame3's instructions by phase (gpurun): one rocprofv3 --pmc pass per frame3_stop cut-off (the
# kernel gives up after that phase, the host reframes with k_frame), each on C3's shape at 10M, so
# that consecutive cut-offs difference into per-phase VALU / SALU / LDS instructions per wave.
#   usage: tools/f3_phase_sq.sh TAG ["bench args"] [lib]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1; A="${2:---workload c3 --entries 10000000} --steps 2 --warmup 1 --quick --no-parity --no-cpu-baseline"; L=$3
O=gpurun_out/$T; mkdir -p $O
[ -n "$L" ] && export SPARKEY_GPU_LIB=$PWD/ablib/$L.so
( while sleep 50; do echo "alive $(date +%T)" >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for s in none 0 1 2 3 4 5; do
  sw=""; [ "$s" != none ] && sw="frame3_stop=$s"
  SPARKEY_DEBUG=$sw timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
    SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d $O/stop_$s -o run -- python3 bench.py $A \
    > $O/stop_$s.log 2>&1 || { tail -5 $O/stop_$s.log; exit 1; }
done
python3 - "$O" <<'EOF' | tee $O/phases.txt
import csv, glob, sys
from collections import defaultdict
d = sys.argv[1]
def per_wave(stop):
    acc = defaultdict(list)
    for f in glob.glob(f"{d}/stop_{stop}/**/*counter_collection.csv", recursive=True):
        per = defaultdict(lambda: defaultdict(float))
        for row in csv.DictReader(open(f)):
            if "k_frame3" not in row["Kernel_Name"]:
                continue
            per[row.get("Dispatch_Id", row.get("Correlation_Id"))][row["Counter_Name"]] += float(row["Counter_Value"])
        for disp in per.values():
            for c, v in disp.items():
                acc[c].append(v)
    m = {c: sum(v) / len(v) for c, v in acc.items()}
    w = m.get("SQ_WAVES", 1.0) or 1.0
    return {c: v / w for c, v in m.items() if c.startswith("SQ_") and c != "SQ_WAVES"}, m.get("GRBM_GUI_ACTIVE", 0.0)
names = {"0": "stage", "1": "screen", "2": "candidates + short walk", "3": "long walk", "4": "heads, resolve, wait",
         "5": "resolve with entry, counts", "none": "hash + entries"}
prev = None
keys = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES"]
print("cut-off".ljust(34), " ".join(k.replace("SQ_", "").ljust(16) for k in keys), "GRBM")
for s in ["0", "1", "2", "3", "4", "5", "none"]:
    pw, g = per_wave(s)
    row = [pw.get(k, 0.0) for k in keys]
    print(f"{s:>4} {names[s]:<29}", " ".join(f"{v:16.1f}" for v in row), f"{g:.0f}")
    if prev is not None:
        print(f"     +{names[s]:<28}", " ".join(f"{a - b:16.1f}" for a, b in zip(row, prev)))
    prev = row
EOF
