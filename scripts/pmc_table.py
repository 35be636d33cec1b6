"""Per-kernel PMC table from rocprofv3 --pmc CSV directories (counter_collection.csv): sums each
counter over the dispatches of a kernel and prints one markdown row per kernel name.

usage: python scripts/pmc_table.py <pmc_dir> [<pmc_dir> ...]

When the FIRST directory also holds a kernel trace (--kernel-trace), the table adds the kernel's
total time in that pass and, with FETCH_SIZE / WRITE_SIZE (kilobytes), the memory-side read / write
rates over that time (counter passes serialise kernels: an in-isolation rate).  The read rate is
2 x FETCH_SIZE: on gfx950 FETCH_SIZE tallies the 128-B requests of a wide coalesced stream at 64 B
(MI355X_MICROARCH.md, "FETCH_SIZE reports exactly 1/2").  With GRBM_GUI_ACTIVE (summed over the 8
XCDs): the effective clock (GRBM / 8 / time) and, with SQ_VALU_MFMA_BUSY_CYCLES (summed over the
1024 SIMDs), the MFMA-busy share = MFMA_BUSY / 1024 / (GRBM / 8).  Counters of different passes
come from different runs of the same program.
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
                if d == sys.argv[1]:
                    disp[k].add(r.get("Dispatch_Id"))
    dur = collections.defaultdict(float)
    for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r.get("Kernel_Name", "?")[:90]] += (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
    names = sorted({c for v in vals.values() for c in v})
    extra = []
    if dur:
        extra = ["ms"] + [x for x, c in (("read TB/s", "FETCH_SIZE"), ("write TB/s", "WRITE_SIZE"),
                                         ("GHz", "GRBM_GUI_ACTIVE")) if c in names]
        if "GRBM_GUI_ACTIVE" in names and "SQ_VALU_MFMA_BUSY_CYCLES" in names:
            extra.append("MFMA busy")
    print("| kernel | dispatches | " + " | ".join(extra + names) + " |")
    print("|---|---:|" + "---:|" * (len(extra) + len(names)))
    key = "SQ_WAVE_CYCLES" if not dur else None
    for k, v in sorted(vals.items(), key=lambda kv: -(dur[kv[0]] if dur else kv[1].get(key, 0))):
        cells = []
        if dur:
            t = dur.get(k, 0.0)
            cells.append(f"{t * 1e3:.3f}")
            for c, f in (("FETCH_SIZE", 2), ("WRITE_SIZE", 1)):
                if c in names:
                    cells.append(f"{f * v.get(c, 0) * 1024 / t / 1e12:.2f}" if t else "-")
            grbm = v.get("GRBM_GUI_ACTIVE", 0) / 8
            if "GRBM_GUI_ACTIVE" in names:
                cells.append(f"{grbm / t / 1e9:.2f}" if t else "-")
            if "MFMA busy" in extra:
                cells.append(f"{100 * v.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / 1024 / grbm:.1f} %" if grbm else "-")
        print(f"| `{k}` | {len(disp[k])} | " + " | ".join(cells + [f"{v.get(c, 0):.4g}" for c in names]) + " |")


if __name__ == "__main__":
    main()
