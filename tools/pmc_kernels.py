"""Per-kernel HBM traffic of a few eager train steps from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE; one counter per run), averaged per launch, with the gfx950
FETCH correction of MI355X_MICROARCH.md (wide coalesced reads report half: doubled).
Fabric-side counts include Infinity-Cache hits, so they bound DRAM bytes from above.

    python tools/pmc_kernels.py FETCH_DIR WRITE_DIR OUT_JSON [--alg kernel=bytes ...]

--alg gives a kernel's algorithmic bytes per launch; the JSON then carries
traffic / algorithmic for it.
"""
import argparse
import collections
import csv
import glob
import json
import os


def load(d, counter):
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(p)) if r["Counter_Name"] == counter]
    acc = collections.defaultdict(list)
    for r in rows:
        acc[r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]].append(float(r["Counter_Value"]))
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("--alg", nargs="*", default=[], help="kernel-substring=bytes per launch")
    ap.add_argument("--zzt-json", default="", help="also write the zz^T kernel's bytes per launch in "
                    "bench.load_traffic's format (C2: N 4096, d 64, 8 graphs, bf16)")
    args = ap.parse_args()
    f, w = load(args.fetch_dir, "FETCH_SIZE"), load(args.write_dir, "WRITE_SIZE")
    alg = {k: float(v) for k, v in (a.split("=") for a in args.alg)}
    out = {"note": "FETCH_SIZE doubled (gfx950 reports half of wide coalesced reads); KiB -> bytes; "
                   "fabric-side counts include Infinity-Cache hits", "kernels": {}}
    for k in sorted(set(f) | set(w)):
        fb = 2.0 * 1024.0 * sum(f.get(k, [0.0])) / max(1, len(f.get(k, [])))
        wb = 1024.0 * sum(w.get(k, [0.0])) / max(1, len(w.get(k, [])))
        e = {"launches": max(len(f.get(k, [])), len(w.get(k, []))), "fetch_bytes": fb,
             "write_bytes": wb, "hbm_bytes_per_launch": fb + wb}
        for sub, b in alg.items():
            if sub in k:
                e["algorithmic_bytes"] = b
                e["traffic_over_algorithmic"] = round((fb + wb) / b, 3)
        out["kernels"][k] = e
    json.dump(out, open(args.out, "w"), indent=1)
    if args.zzt_json:
        k, e = next((k, e) for k, e in out["kernels"].items() if "zzt_dense" in k)
        json.dump({"kernel": k, "n_nodes": 4096, "latent": 64, "graphs": 8, "dtype": "bf16",
                   "launches": e["launches"], "fetch_bytes": e["fetch_bytes"], "write_bytes": e["write_bytes"],
                   "hbm_bytes_per_launch": e["hbm_bytes_per_launch"],
                   "source": "tools/pmc_kernels.py over rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of "
                             "tools/prof_step.py --steps 3 (eager C2 steps); FETCH doubled (gfx950)"},
                  open(args.zzt_json, "w"), indent=1)
    top = sorted(out["kernels"].items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:12]
    for k, e in top:
        print(f"{e['hbm_bytes_per_launch'] / 1e6:9.2f} MB  {k[-60:]}  {e.get('traffic_over_algorithmic', '')}")


if __name__ == "__main__":
    main()
