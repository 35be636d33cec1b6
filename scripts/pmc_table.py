"""Per-kernel PMC table from rocprofv3 --pmc CSV directories (counter_collection.csv): sums each
counter over the dispatches of a kernel and prints one markdown row per kernel name.

usage: python scripts/pmc_table.py <pmc_dir> [<pmc_dir> ...]
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
    names = sorted({c for v in vals.values() for c in v})
    print("| kernel | dispatches | " + " | ".join(names) + " |")
    print("|---|---:|" + "---:|" * len(names))
    for k, v in sorted(vals.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        print(f"| `{k}` | {len(disp[k])} | " + " | ".join(f"{v.get(c, 0):.4g}" for c in names) + " |")


if __name__ == "__main__":
    main()
