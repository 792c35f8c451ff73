"""Summarise rocprofv3 outputs (kernel stats + PMC passes) into one JSON under profiles/.

    python tools/pmc_summary.py gpurun_out/prof profiles/r01_pmc_summary.json

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE counts 64 B per 128-B
request of a wide coalesced stream, i.e. half the bytes (MI355X_MICROARCH.md "HBM"): the read
side is doubled here; WRITE_SIZE is taken as is.
"""
import csv
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("sk::", "")
    return n.split("<")[0]


def read_counters(path):
    acc = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return acc
    with open(path) as f:
        for row in csv.DictReader(f):
            acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def main(src, dst, workload=None):
    stats = {}
    with open(os.path.join(src, "trace", "run_kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            k = short(row["Name"])
            s = stats.setdefault(k, {"calls": 0, "total_ns": 0.0})
            s["calls"] += int(row["Calls"])
            s["total_ns"] += float(row["TotalDurationNs"])
    for s in stats.values():
        s["avg_us"] = s["total_ns"] / s["calls"] / 1e3
    fetch = read_counters(os.path.join(src, "fetch", "run_counter_collection.csv"))
    write = read_counters(os.path.join(src, "write", "run_counter_collection.csv"))
    sq = read_counters(os.path.join(src, "sq", "run_counter_collection.csv"))
    out = {"kernels": {}, "per_launch_hbm_bytes": {}}
    for k, s in sorted(stats.items(), key=lambda kv: -kv[1]["total_ns"]):
        rec = dict(s)
        f = fetch.get(k, {}).get("FETCH_SIZE")
        w = write.get(k, {}).get("WRITE_SIZE")
        if f:
            rec["fetch_bytes_corrected"] = 2 * 1024 * sum(f) / len(f)
        if w:
            rec["write_bytes"] = 1024 * sum(w) / len(w)
        if f and w:
            rec["hbm_bytes"] = rec["fetch_bytes_corrected"] + rec["write_bytes"]
        for c, vals in sq.get(k, {}).items():
            rec[c] = sum(vals) / len(vals)
        out["kernels"][k] = rec
    # stage name (bench.py) -> kernels in that stage
    stage_kernels = {"frame": ["k_frame", "k_frame_uniform", "k_frame2", "k_frame3", "k_frame_lane", "k_frame_lane_act",
                               "k_frame_lane_flags"], "frame_uniform": ["k_frame_uniform"],
                     "partition": ["k_part1_hist", "k_part1_scatter", "k_part1_regions", "k_part2", "k_part2s", "k_part2st", "k_part2d",
                                   "k_part2f", "k_part2f_direct", "k_part2_sub", "k_scan_tiles"],
                     "partition_regions": ["k_part2", "k_part2s", "k_part2st", "k_part2d", "k_part2f", "k_part2f_direct", "k_part2_sub"],
                     "place": ["k_place_lds", "k_place_reg", "k_place_reg_persist", "k_place", "k_place_fix"],
                     "stats": ["k_stats", "k_stats_final", "k_stats_folded"],
                     "summary": ["k_summary", "k_carry"], "verify": ["k_verify_pairs"]}
    for st, ks in stage_kernels.items():
        tot = 0.0
        ok = False
        for k in ks:
            r = out["kernels"].get(k)
            if r and "hbm_bytes" in r:
                tot += r["hbm_bytes"]
                ok = True
        if ok:
            out["per_launch_hbm_bytes"][st] = tot
    # the whole build: every kernel's bytes per dispatch times its dispatches per build (one k_build_init
    # a single-GPU build; a sharded rank counts its frame launches)
    ref = next((k for k in ("k_frame_uniform", "k_frame3", "k_frame", "k_build_init") if k in out["kernels"]), None)
    if ref and all("hbm_bytes" in r for k, r in out["kernels"].items()
                   if k.startswith("k_") and r["total_ns"] > 0.01 * out["kernels"][ref]["total_ns"]):
        nb = out["kernels"][ref]["calls"]
        # (the library's kernels only: torch's data generation and runtime copies are not the build; a
        #  kernel launched fewer times than the framing kernel belongs to another leg of the run, such
        #  as bench.py's general-framing comparison, and is left out)
        out["per_launch_hbm_bytes"]["build"] = sum(r.get("hbm_bytes", 0.0) * max(1, round(r["calls"] / nb))
                                                   for k, r in out["kernels"].items()
                                                   if k.startswith("k_") and r["calls"] >= nb)
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    if workload:  # merge: one summary file holds every workload's counters
        try:
            with open(dst) as f:
                prev = json.load(f)
        except (OSError, ValueError):
            prev = {}
        by = prev.get("per_launch_hbm_bytes_by_workload", {})
        kern = prev.get("kernels_by_workload", {})
        by[workload] = out["per_launch_hbm_bytes"]
        kern[workload] = out["kernels"]
        out = {"per_launch_hbm_bytes_by_workload": by, "kernels_by_workload": kern}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    for k, r in (out.get("kernels") or out["kernels_by_workload"][workload]).items():
        print(f"{k:28s} {r['avg_us']:9.1f} us  hbm={r.get('hbm_bytes', 0)/1e6:9.1f} MB  "
              f"valu={r.get('SQ_INSTS_VALU', 0):.3g} lds={r.get('SQ_INSTS_LDS', 0):.3g}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
