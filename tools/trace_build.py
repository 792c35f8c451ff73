"""Timeline of one build from a rocprofv3 kernel trace: kernels between the last two launches of a
marker kernel, with the idle gaps before each (tools/trace_build.py TRACE.csv [MARKER])."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2] if len(sys.argv) > 2 else "frame_uniform"
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
t0 = int(rows[a]["Start_Timestamp"])
busy, prev_end, gaps = 0, t0, 0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = max(0, s - prev_end) / 1000
    gaps += gap
    print(f"{(s - t0) / 1000:8.1f} gap {gap:7.1f} dur {(e - s) / 1000:7.1f}  {r['Kernel_Name'][:80]}")
    busy += e - s
    prev_end = max(prev_end, e)
span = (int(rows[b]["Start_Timestamp"]) - t0) / 1000
print(f"busy {busy / 1000:.1f} us, gaps {gaps + max(0, int(rows[b]['Start_Timestamp']) - prev_end) / 1000:.1f} us, span {span:.1f} us")
