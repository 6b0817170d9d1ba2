"""Summarise rocprofv3 --pmc counter CSVs (tools/pmc_sq.sh) of one kernel: the last
dispatch whose name contains KERNEL_SUBSTR, per counter, plus derived per-SIMD cycles.

    python tools/pmc_sq.py DIR KERNEL_SUBSTR
"""
import csv
import glob
import json
import os
import sys


def main():
    d, k = sys.argv[1], sys.argv[2]
    sub = {"zzt_dense": "zzt_dense_bf16", "zzt_dense_v3": "zzt_dense_bf16_v3"}.get(k, k)
    cnt = {}
    for path in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        last = {}
        for r in csv.DictReader(open(path)):
            if sub in r["Kernel_Name"]:
                key = (r["Counter_Name"])
                disp = int(r.get("Dispatch_Id", 0) or 0)
                prev = last.get(key)
                if prev is None or disp > prev[0]:
                    last[key] = (disp, 0.0, r["Kernel_Name"])
                if disp == last[key][0]:
                    last[key] = (disp, last[key][1] + float(r["Counter_Value"]), r["Kernel_Name"])
        for key, (_, v, name) in last.items():
            cnt[key] = v
            cnt["_kernel"] = name[:120]
    out = {"counters": cnt}
    wc = cnt.get("SQ_WAVE_CYCLES")
    if wc:
        out["derived"] = {
            "frac_active_any": cnt.get("SQ_ACTIVE_INST_ANY", 0) / wc,
            "frac_active_valu": cnt.get("SQ_ACTIVE_INST_VALU", 0) / wc,
            "frac_wait_any": cnt.get("SQ_WAIT_ANY", 0) / wc,
            "frac_wait_inst_any": cnt.get("SQ_WAIT_INST_ANY", 0) / wc,
            "note": "fractions of wave-cycles (SQ_*_CYCLES / ACTIVE / WAIT are quad-cycles)",
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
