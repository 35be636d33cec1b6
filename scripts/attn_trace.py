"""Every causal prefill-attention launch of a rocprofv3 kernel trace: duration, grid (pair groups x
heads x sequences) and the kernel before it -> markdown table (where the in-model attention time goes)."""
import csv
import os
import sys


def main(d, prefix, out):
    rows = []
    with open(os.path.join(d, f"{prefix}_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            rows.append(r)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    lines = ["| # | us | grid x | grid y | grid z | wg size | previous kernel |", "|---:|---:|---:|---:|---:|---:|---|"]
    n = 0
    for i, r in enumerate(rows):
        if "flash_d128" not in r.get("Kernel_Name", ""):
            continue
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        gx, gy, gz = (r.get(f"Grid_Size_{a}", r.get(f"Grid_Size{a}", "?")) for a in "XYZ")
        wg = r.get("Workgroup_Size_X", r.get("Workgroup_Size", "?"))
        prev = rows[i - 1].get("Kernel_Name", "")[:60] if i else ""
        lines.append(f"| {n} | {us:.1f} | {gx} | {gy} | {gz} | {wg} | `{prev}` |")
        n += 1
    with open(out, "w") as f:
        f.write("# prefill attention launches\n\n" + "\n".join(lines) + "\n")
    print(f"{n} launches -> {out}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
