"""Print the per-dispatch timeline of the last train step in a rocprofv3 kernel trace.

    python tools/step_timeline.py gpurun_out/prof/run_kernel_trace.csv
"""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # a step ends with its last Adam launch (graph-latent plans run several Adam passes),
    # or with the final reduction when Adam rides in it (ABI 16)
    key = "adam" if any("adam" in r["Kernel_Name"] for r in rows) else "reduce_kernel"
    ad = [key in r["Kernel_Name"] for r in rows]
    ends = [i for i in range(len(rows)) if ad[i] and (i + 1 == len(rows) or not ad[i + 1])]
    a, b = ends[-2] + 1, ends[-1] + 1
    t0 = int(rows[a]["Start_Timestamp"])
    busy = 0
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        n = r["Kernel_Name"].replace("snd::(anonymous namespace)::", "").replace("_ZN3snd12_GLOBAL__N_1", "")
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.2f}  grid {r['Grid_Size_X']:>7}x{r['Grid_Size_Y']:>3}"
              f"x{r.get('Grid_Size_Z', '1'):>3} lds {r['LDS_Block_Size']:>6} vgpr {r['VGPR_Count']:>3}/{r['Accum_VGPR_Count']:>3}  {n[:70]}")
    end = int(rows[b - 1]["End_Timestamp"])
    print(f"step span {(end - t0) / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us, {b - a} launches")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv")
