#!/usr/bin/env python
"""Attribute rocprofv3 kernel time to the engine's roctx phase ranges.

    DAB_ROCTX=1 rocprofv3 --marker-trace --kernel-trace -d OUT -o bench --output-format csv -- python bench.py ...
    python scripts/roctx_attribution.py OUT/bench_marker_api_trace.csv OUT/bench_kernel_trace.csv [summary.md]

A kernel belongs to the latest range that STARTED before the kernel started (every engine phase ends
in a host sync, so a phase's kernels finish before the next phase's range opens).
"""
import bisect
import csv
import sys
from collections import defaultdict


def main():
    markers, kernels = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    ranges = []
    with open(markers) as f:
        for r in csv.DictReader(f):
            ranges.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]))
    ranges.sort()
    starts = [r[0] for r in ranges]
    per = defaultdict(lambda: [0, 0.0, defaultdict(float)])
    wall = defaultdict(float)
    for s, e, name in ranges:
        wall[name] += (e - s) / 1e6
    first = starts[0] if starts else 0
    with open(kernels) as f:
        for k in csv.DictReader(f):
            ks, ke = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
            if ks < first:
                continue  # setup before the first phase
            i = bisect.bisect_right(starts, ks) - 1
            name = ranges[i][2]
            rec = per[name]
            rec[0] += 1
            rec[1] += (ke - ks) / 1e6
            rec[2][k["Kernel_Name"][:90]] += (ke - ks) / 1e6
    lines = ["| phase (roctx range) | ranges | host wall ms | kernels | kernel ms | top kernels (ms) |", "|---|---:|---:|---:|---:|---|"]
    nr = defaultdict(int)
    for _, _, n in ranges:
        nr[n] += 1
    for name, (cnt, ms, ks) in sorted(per.items(), key=lambda x: -x[1][1]):
        top = sorted(ks.items(), key=lambda x: -x[1])[:3]
        tops = "; ".join(f"`{n.split('(')[0][:60]}` {v:.1f}" for n, v in top)
        lines.append(f"| {name} | {nr[name]} | {wall[name]:.1f} | {cnt} | {ms:.1f} | {tops} |")
    text = "\n".join(lines)
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
