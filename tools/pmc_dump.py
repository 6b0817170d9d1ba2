"""Per-kernel average of every counter in a rocprofv3 --pmc output directory.

    python tools/pmc_dump.py DIR [--kernels sub1,sub2]
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernels", default="")
    args = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in glob.glob(os.path.join(args.dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    subs = [s for s in args.kernels.split(",") if s]
    for k in sorted(acc):
        if subs and not any(s in k for s in subs):
            continue
        print(k, {c: round(sum(v) / len(v), 1) for c, v in sorted(acc[k].items())})


if __name__ == "__main__":
    main()
