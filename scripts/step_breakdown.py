"""Per-step kernel breakdown from a rocprofv3 --kernel-trace CSV.

usage: python scripts/step_breakdown.py <prof_dir> <prefix> [--out out.md]

A model step starts with ``embed_gather_kernel`` (token embedding gather) in both prefill and decode.
The last step whose window contains ``flash_fwd`` is reported as the prefill step, the last window
containing ``paged_decode`` as the decode step: kernel time aggregated by name, the GPU-busy share of
the step's span, and the mean inter-kernel gap (launch / graph overhead).
"""
import csv
import os
import sys
from collections import defaultdict


# Llama prefill attention launches (the 32x32 D=128 kernel, or the 16x16 one it replaced); the
# encoder's D=64 flash launches belong to the query-embedding step, not to a prefill
def _is_prefill_attn(name: str) -> bool:
    return "flash_d128" in name or "flash_fwd_kernel<128" in name


def short(name: str) -> str:
    name = name.replace("void ", "")
    if name.startswith("Cijk") or name.startswith("Custom_Cijk"):
        mt = [p for p in name.split("_") if p.startswith("MT")]
        return "hipBLASLt " + (mt[0] if mt else name[:40])
    return name.split("(")[0][:70]


def window_table(win, title):
    busy = sum(e - s for s, e, _ in win)
    span = win[-1][1] - win[0][0]
    gaps = [max(0, win[i + 1][0] - win[i][1]) for i in range(len(win) - 1)]
    agg = defaultdict(lambda: [0, 0])
    for s, e, n in win:
        a = agg[short(n)]
        a[0] += 1
        a[1] += e - s
    lines = [f"## {title}", "",
             f"{len(win)} kernels, span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms "
             f"({100.0 * busy / max(span, 1):.1f} %), mean gap {sum(gaps) / max(1, len(gaps)) / 1e3:.2f} us", "",
             "| kernel | calls | total us | avg us | % of busy |", "|---|---:|---:|---:|---:|"]
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"| `{k}` | {c} | {t / 1e3:.1f} | {t / 1e3 / c:.2f} | {100.0 * t / max(busy, 1):.1f} |")
    return lines + [""]


def main():
    d, prefix = sys.argv[1], sys.argv[2]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    rows = []
    with open(os.path.join(d, f"{prefix}_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "embed_gather_kernel" in r[2]] + [len(rows)]
    steps = [rows[starts[i]:starts[i + 1]] for i in range(len(starts) - 1)]
    lines = [f"# per-step kernel breakdown: {prefix}", ""]
    dec = [s for s in steps if any("paged_decode" in n for _, _, n in s) and not any(_is_prefill_attn(n) for _, _, n in s)]
    mixed = [s for s in steps if any(_is_prefill_attn(n) for _, _, n in s) and any("paged_decode" in n for _, _, n in s)]
    pre = [s for s in steps if any(_is_prefill_attn(n) for _, _, n in s) and s not in mixed]
    if mixed:
        spans = sorted((s[-1][1] - s[0][0]) / 1e6 for s in mixed)
        med = min(mixed, key=lambda s: abs((s[-1][1] - s[0][0]) / 1e6 - spans[len(spans) // 2]))
        lines += window_table(med, "median mixed step (prompt chunks + decode rows in one forward)")
        lines += [f"mixed steps: {len(mixed)}, median span {spans[len(spans) // 2]:.3f} ms", ""]
    if pre:
        big = max(pre, key=lambda s: s[-1][1] - s[0][0])
        lines += window_table(big, "largest prefill step")
        tot = sum(s[-1][1] - s[0][0] for s in pre) / 1e6
        busy = sum(e - b for s in pre for b, e, _ in s) / 1e6
        lines += [f"prefill steps: {len(pre)}, span {tot:.1f} ms, kernels busy {busy:.1f} ms", ""]
    if dec:
        lines += window_table(dec[-1], "last decode step")
        if len(dec) > 1:
            spans = sorted((s[-1][1] - s[0][0]) / 1e6 for s in dec)
            lines += [f"decode steps: {len(dec)}, median span {spans[len(spans) // 2]:.3f} ms", ""]
    text = "\n".join(lines)
    print(text)
    if out:
        open(out, "w").write(text + "\n")


if __name__ == "__main__":
    main()
