"""Convert rocprofv3 FETCH_SIZE / WRITE_SIZE counter CSVs of the fused zz^T
kernel into profiles/<tag>_pmc_zzt.json (HBM bytes per launch).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half
the bytes of wide coalesced streaming reads (TCC_EA0_RDREQ x 64 B for 128-B
requests) -> doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  Both are
in KiB.  Infinity-Cache hits are counted (fabric-side requests), so this is an
upper bound on DRAM bytes.

    python tools/pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON n_nodes latent graphs dtype
"""
import csv
import json
import sys


def per_launch(path, counter, kernel="zzt_dense"):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return sum(vals) / len(vals), len(vals)


def main():
    fetch_csv, write_csv, out, n, d, b, dtype = sys.argv[1:8]
    f, nf = per_launch(fetch_csv, "FETCH_SIZE")
    w, nw = per_launch(write_csv, "WRITE_SIZE")
    fetch_b = 2.0 * f * 1024.0
    write_b = w * 1024.0
    j = {"kernel": "zzt_dense_bf16 (fused z z^T + CE)", "n_nodes": int(n), "latent": int(d),
         "graphs": int(b), "dtype": dtype, "launches_averaged": min(nf, nw),
         "fetch_size_kib_raw": f, "write_size_kib_raw": w,
         "fetch_bytes_corrected": fetch_b, "write_bytes": write_b,
         "hbm_bytes_per_launch": fetch_b + write_b,
         "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 reports half of wide "
                 "coalesced reads); fabric-side counts include Infinity-Cache hits"}
    json.dump(j, open(out, "w"), indent=1)
    print(json.dumps(j))


if __name__ == "__main__":
    main()
