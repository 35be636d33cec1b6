"""Per-kernel PMC table from rocprofv3 --pmc CSV directories (counter_collection.csv): sums each
counter over the dispatches of a kernel and prints one markdown row per kernel name.

usage: python scripts/pmc_table.py <pmc_dir> [<pmc_dir> ...]

When the FIRST directory also holds a kernel trace (--kernel-trace), the table adds the kernel's
total time in that pass and, with FETCH_SIZE / WRITE_SIZE (kilobytes), the HBM-side read / write
rates over that time (counter passes serialise kernels: an in-isolation rate).
"""
import collections
import csv
import glob
import os
import sys


def main():
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r.get("Kernel_Name", "?")[:90]
                vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((d, r.get("Dispatch_Id")))
    dur = collections.defaultdict(float)
    for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r.get("Kernel_Name", "?")[:90]] += (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
    names = sorted({c for v in vals.values() for c in v})
    extra = []
    if dur:
        extra = ["ms"] + [x for x, c in (("read TB/s", "FETCH_SIZE"), ("write TB/s", "WRITE_SIZE")) if c in names]
    print("| kernel | dispatches | " + " | ".join(extra + names) + " |")
    print("|---|---:|" + "---:|" * (len(extra) + len(names)))
    key = "SQ_WAVE_CYCLES" if not dur else None
    for k, v in sorted(vals.items(), key=lambda kv: -(dur[kv[0]] if dur else kv[1].get(key, 0))):
        cells = []
        if dur:
            t = dur.get(k, 0.0)
            cells.append(f"{t * 1e3:.3f}")
            for c in ("FETCH_SIZE", "WRITE_SIZE"):
                if c in names:
                    cells.append(f"{v.get(c, 0) * 1024 / t / 1e12:.2f}" if t else "-")
        print(f"| `{k}` | {len(disp[k])} | " + " | ".join(cells + [f"{v.get(c, 0):.4g}" for c in names]) + " |")


if __name__ == "__main__":
    main()
