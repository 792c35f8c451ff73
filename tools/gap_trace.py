"""Kernel timeline of a rocprofv3 --kernel-trace run: per-build kernel durations and the idle gaps
between kernels (host launch overhead), from run_kernel_trace.csv.

    python tools/gap_trace.py gpurun_out/TAG/trace/run_kernel_trace.csv FIRST_KERNEL
FIRST_KERNEL: a substring of the kernel that starts every build (e.g. k_build_init)."""
import csv
import sys
from collections import defaultdict


def main(path, first):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")))
    rows.sort()
    builds, cur = [], []
    for r in rows:
        if first in r[2] and cur:
            builds.append(cur)
            cur = []
        cur.append(r)
    if cur:
        builds.append(cur)
    builds = [b for b in builds if first in b[0][2]]
    stats = defaultdict(list)
    for b in builds[2:]:  # (warmup)
        span = b[-1][1] - b[0][0]
        busy = sum(e - s for s, e, _ in b)
        stats["span_us"].append(span / 1e3)
        stats["busy_us"].append(busy / 1e3)
        for (s0, e0, n0), (s1, e1, n1) in zip(b, b[1:]):
            stats[f"gap {n0.split('::')[-1][:24]} -> {n1.split('::')[-1][:24]}"].append((s1 - e0) / 1e3)
    for i in range(2, len(builds) - 1):
        stats["between_builds_us"].append((builds[i + 1][0][0] - builds[i][-1][1]) / 1e3)
    for k, v in stats.items():
        v = sorted(v)
        print(f"{k:70s} median {v[len(v) // 2]:8.2f}  (n {len(v)})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
