"""Per-kernel-slot timing of the decode layer from a rocprofv3 --kernel-trace CSV.

usage: python scripts/decode_layer_profile.py <prof_dir> <prefix> [--steps N] [--out file.md]

Decode steps are the windows between ``embed_gather_kernel`` launches that contain paged decode
attention and no flash prefill.  Inside a step the layers are cut at each paged-decode launch; each
kernel gets a slot = its offset from the layer's attention kernel, and the table reports per slot the
median duration and the median gap before it, over every layer of the last N decode steps."""
import csv
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from step_breakdown import short  # noqa: E402


# Llama prefill attention launches (the 32x32 D=128 kernel, or the 16x16 one it replaced); the
# encoder's D=64 flash launches belong to the query-embedding step, not to a prefill
def _is_prefill_attn(name: str) -> bool:
    return "flash_d128" in name or "flash_fwd_kernel<128" in name


def main():
    d, prefix = sys.argv[1], sys.argv[2]
    nsteps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 20
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    rows = []
    with open(os.path.join(d, f"{prefix}_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "embed_gather_kernel" in r[2]] + [len(rows)]
    steps = [rows[starts[i]:starts[i + 1]] for i in range(len(starts) - 1)]
    dec = [s for s in steps if any("paged_decode" in n for _, _, n in s) and not any(_is_prefill_attn(n) for _, _, n in s)]
    dec = dec[-nsteps:]
    slots = defaultdict(lambda: {"dur": [], "gap": [], "name": ""})
    spans = []
    for s in dec:
        spans.append((s[-1][1] - s[0][0]) / 1e6)
        att = [i for i, (_, _, n) in enumerate(s) if "paged_decode" in n]
        for li in range(1, len(att) - 1):
            a, b = att[li], att[li + 1]
            for i in range(a, b):
                st, en, n = s[i]
                slot = slots[i - a]
                slot["dur"].append((en - st) / 1e3)
                slot["gap"].append(max(0, st - s[i - 1][1]) / 1e3)
                slot["name"] = short(n)
    lines = [f"# decode layer, per kernel slot ({len(dec)} decode steps, median step span "
             f"{statistics.median(spans):.3f} ms)", "",
             "| slot | kernel | median us | median gap before us |", "|---:|---|---:|---:|"]
    tot = 0.0
    for k in sorted(slots):
        v = slots[k]
        md = statistics.median(v["dur"])
        tot += md + statistics.median(v["gap"])
        lines.append(f"| {k} | `{v['name']}` | {md:.2f} | {statistics.median(v['gap']):.2f} |")
    lines += ["", f"layer total (medians incl. gaps): {tot:.1f} us"]
    text = "\n".join(lines) + "\n"
    if out:
        with open(out, "w") as f:
            f.write(text)
    print(text)


if __name__ == "__main__":
    main()
