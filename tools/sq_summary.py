"""Per-wave SQ counters of one kernel from tools/r05_sq.sh's two rocprofv3 --pmc passes.

    python tools/sq_summary.py gpurun_out/TAG k_frame3
Counters are summed over a dispatch's XCDs and averaged over the dispatches; per-wave figures divide
by SQ_WAVES, resident waves per SIMD = SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE * 1024 SIMDs / 8 XCDs)...
(SQ_WAVE_CYCLES counts in units of 4 cycles on gfx9, as do the WAIT/ACTIVE counters; figures below
are reported in those units, their ratios are what matter)."""
import csv
import glob
import sys
from collections import defaultdict


def load(d, kernel):
    acc = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = defaultdict(lambda: defaultdict(float))
        for row in csv.DictReader(open(f)):
            if kernel not in row["Kernel_Name"]:
                continue
            per[row.get("Dispatch_Id", row.get("Correlation_Id"))][row["Counter_Name"]] += float(row["Counter_Value"])
        for disp in per.values():
            for c, v in disp.items():
                acc[c].append(v)
    return {c: sum(v) / len(v) for c, v in acc.items()}


def main(d, kernel):
    a = load(f"{d}/p1", kernel)
    b = load(f"{d}/p2", kernel)
    c = {**b, **a}
    w = c.get("SQ_WAVES", 1.0)
    print(f"{kernel}: waves {w:.0f}  GRBM_GUI_ACTIVE {c.get('GRBM_GUI_ACTIVE', 0):.0f}")
    for k in sorted(c):
        print(f"  {k:24s} {c[k]:16.0f}  per wave {c[k] / w:10.1f}")
    wc = c.get("SQ_WAVE_CYCLES", 0)
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA",
                  "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if k in c:
                print(f"  {k:24s} share of wave cycles {c[k] / wc:.3f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
