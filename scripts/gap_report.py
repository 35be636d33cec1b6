"""GPU idle gaps in a rocprofv3 kernel trace: where the device waits for the host.

usage: python scripts/gap_report.py <prof_dir> <prefix> [--min-us 50] [--top 30] [--last-ms T] [--out gaps.md]

Sorts the kernels by start time and lists every gap between the end of one kernel (running max of
end stamps, so overlapping kernels don't create false gaps) and the start of the next one that is
at least ``--min-us`` long.  The kernels on both sides identify the host step that stalled the GPU
(prefill chunk hand-off, the prefill -> decode switch, batch boundaries, ...).  ``--last-ms T``
keeps the last T ms of the trace (e.g. the timed batch of ``bench.py --steps 1 --no-fast-steps``).
"""
import csv
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    return name.replace("void ", "").split("(")[0][:60]


def main():
    d, prefix = sys.argv[1], sys.argv[2]
    arg = lambda k, dflt: type(dflt)(sys.argv[sys.argv.index(k) + 1]) if k in sys.argv else dflt  # noqa: E731
    min_us, top, out, last = arg("--min-us", 50.0), arg("--top", 30), arg("--out", ""), arg("--last-ms", 0.0)
    rows = []
    with open(os.path.join(d, f"{prefix}_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")))
    rows.sort()
    if last > 0:
        t_end = max(e for _, e, _ in rows)
        rows = [r for r in rows if r[0] >= t_end - last * 1e6]
    t0 = rows[0][0]
    gaps = []
    end, prev = rows[0][1], rows[0][2]
    for s, e, n in rows[1:]:
        if s - end >= min_us * 1e3:
            gaps.append(((s - end) / 1e3, (end - t0) / 1e6, prev, n))
        if e > end:
            end, prev = e, n
    by_pair = defaultdict(lambda: [0, 0.0])
    for g, _, a, b in gaps:
        k = (short(a), short(b))
        by_pair[k][0] += 1
        by_pair[k][1] += g
    span = (end - t0) / 1e6
    lines = [f"# GPU idle gaps >= {min_us:g} us: {prefix}", "",
             f"{len(rows)} kernels over {span:.1f} ms; {len(gaps)} gaps, {sum(g for g, *_ in gaps) / 1e3:.1f} ms idle", "",
             "## by (kernel before, kernel after)", "",
             "| before | after | gaps | total ms |", "|---|---|---:|---:|"]
    for (a, b), (c, t) in sorted(by_pair.items(), key=lambda kv: -kv[1][1])[:top]:
        lines.append(f"| `{a}` | `{b}` | {c} | {t / 1e3:.2f} |")
    lines += ["", f"## largest {top}", "", "| at ms | gap us | before | after |", "|---:|---:|---|---|"]
    for g, at, a, b in sorted(gaps, key=lambda x: -x[0])[:top]:
        lines.append(f"| {at:.1f} | {g:.0f} | `{short(a)}` | `{short(b)}` |")
    text = "\n".join(lines) + "\n"
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
