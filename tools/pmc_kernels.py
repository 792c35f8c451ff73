"""Mean per-dispatch value of every counter in rocprofv3 --pmc CSVs, per kernel.

    python tools/pmc_kernels.py gpurun_out/pmcp/a/run_counter_collection.csv [...] [--kernels k_place_lds,k_part2]
"""
import csv
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "").replace("sk::", "").split("<")[0]


def main(argv):
    want = None
    paths = []
    for a in argv:
        if a.startswith("--kernels="):
            want = set(a.split("=", 1)[1].split(","))
        else:
            paths.append(a)
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        with open(p) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                if want and k not in want:
                    continue
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print(f"  {c:24s} {sum(v) / len(v):16.0f}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1:])
