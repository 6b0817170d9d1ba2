"""Join rocprofv3 --pmc passes of tools/prof_step.py into a per-kernel table
for the last step (dispatch order), plus derived ratios.

    python tools/pmc_step.py gpurun_out/pmcs1 gpurun_out/pmcs2 ...
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return None
    rows = list(csv.DictReader(open(f[0])))
    by = defaultdict(dict)
    names = {}
    for r in rows:
        did = int(r["Dispatch_Id"])
        by[did][r["Counter_Name"]] = by[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[did] = r["Kernel_Name"]
    ids = sorted(by)
    # last step = dispatches after the second-to-last adam kernel
    ad = [i for i in ids if "adam" in names[i]]
    lo = ad[-2] if len(ad) >= 2 else ids[0] - 1
    step = [i for i in ids if lo < i <= ad[-1]]
    return [(names[i], by[i]) for i in step]


def short(n):
    n = n.replace("snd::(anonymous namespace)::", "").replace("_ZN3snd12_GLOBAL__N_1", "")
    return n[:48]


def main():
    passes = [p for p in (load(d) for d in sys.argv[1:]) if p]
    n = min(len(p) for p in passes)
    table = []
    for k in range(n):
        row = {}
        for p in passes:
            row.update(p[k][1])
        table.append((passes[0][k][0], row))
    keys = sorted({c for _, r in table for c in r})
    print("kernel".ljust(50) + "".join(c[:14].rjust(15) for c in keys))
    for name, r in table:
        print(short(name).ljust(50) + "".join(f"{r.get(c, float('nan')):15.4g}" for c in keys))


if __name__ == "__main__":
    main()
