"""HBM traffic of the window SpMM on bench.py's secondary-roofline batch, from two
rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of tools/ab_spmm_win.py, in the format
bench.load_spmm_traffic reads (profiles/*pmc_spmm_win.json).

    python tools/pmc_spmm_win.py FETCH_DIR WRITE_DIR OUT_JSON --nnz 16266176 --beta 258
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pmc_kernels import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("--nnz", type=int, required=True)
    ap.add_argument("--beta", type=int, required=True)
    ap.add_argument("--rows", type=int, default=256 * 4096)
    args = ap.parse_args()
    f, w = load(args.fetch_dir, "FETCH_SIZE"), load(args.write_dir, "WRITE_SIZE")
    k = next(k for k in f if "spmm_win_kernel" in k)
    fk = sum(f[k]) / len(f[k])                      # KiB per launch
    wk = sum(w[k]) / len(w[k])
    rd, wr = int(2 * 1024 * fk), int(1024 * wk)
    alg = 4 * (args.rows + 1) + 4 * args.nnz + 2 * 2 * args.rows * 64
    out = {
        "kernel": f"{k} (snd_csr_spmm_bf16_window)",
        "workload": (f"bench secondary roofline: A @ H, width 64, 256 graphs block-diagonal (8 RGGs N=4096 x 32 "
                     f"copies), {args.nnz} nnz, RCM schedule, beta {args.beta}, 1096-row LDS ring"),
        "command": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (one pass each) -- python tools/ab_spmm_win.py "
                   "--flags 0 --rounds 1",
        "launches": len(f[k]),
        "fetch_size_kib_per_launch": round(fk, 1),
        "write_size_kib_per_launch": round(wk, 1),
        "correction": "gfx950: FETCH_SIZE x2 for 16-B-per-lane streaming reads (MI355X_MICROARCH.md HBM section); "
                      "WRITE_SIZE exact for 16-B stores",
        "hbm_read_bytes_per_launch": rd,
        "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr,
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": round((rd + wr) / alg, 3),
    }
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
