"""Summarise a rocprofv3 --kernel-trace --stats CSV directory into a small markdown table.

usage: python scripts/prof_summary.py <prof_dir> <prefix> <out.md> [--drop-trace]
Also reports GPU-busy time (union of kernel intervals) vs the traced wall span.
"""
import csv
import os
import sys


# Llama prefill attention launches (the 32x32 D=128 kernel, or the 16x16 one it replaced); the
# encoder's D=64 flash launches belong to the query-embedding step, not to a prefill
def _is_prefill_attn(name: str) -> bool:
    return "flash_d128" in name or "flash_fwd_kernel<128" in name


def main():
    d, prefix, out = sys.argv[1], sys.argv[2], sys.argv[3]
    stats = list(csv.DictReader(open(os.path.join(d, f"{prefix}_kernel_stats.csv"))))
    tot = sum(float(r["TotalDurationNs"]) for r in stats)
    lines = [f"# rocprofv3 kernel stats: {prefix}", "", f"total kernel time: {tot / 1e6:.1f} ms", ""]
    tpath = os.path.join(d, f"{prefix}_kernel_trace.csv")
    if os.path.exists(tpath):
        iv, named = [], []
        with open(tpath) as f:
            for r in csv.DictReader(f):
                iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
                named.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")))
        iv.sort()
        named.sort()
        # decode window: after the last prefill attention kernel, from the first to the last paged
        # decode kernel -> GPU busy share and inter-kernel gaps inside the graph replays
        last_pf = max((i for i, k in enumerate(named) if _is_prefill_attn(k[2])), default=-1)
        dec = [k for k in named[last_pf + 1:]]
        di = [i for i, k in enumerate(dec) if "paged_decode" in k[2]]
        if di:
            win = dec[di[0]:di[-1] + 1]
            wbusy = sum(e - s for s, e, _ in win)
            wspan = win[-1][1] - win[0][0]
            gaps = [max(0, win[i + 1][0] - win[i][1]) for i in range(len(win) - 1)]
            lines += [f"decode window (last step): {len(win)} kernels, busy {wbusy / 1e6:.2f} ms of "
                      f"{wspan / 1e6:.2f} ms ({100.0 * wbusy / max(wspan, 1):.1f} %), mean gap "
                      f"{(sum(gaps) / max(1, len(gaps))) / 1e3:.2f} us, {len(di)} paged-decode launches", ""]
        busy, cur_s, cur_e = 0, None, None
        for s, e in iv:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        span = iv[-1][1] - iv[0][0] if iv else 0
        lines += [f"kernels traced: {len(iv)}; GPU busy {busy / 1e6:.1f} ms of {span / 1e6:.1f} ms span "
                  f"({100.0 * busy / max(span, 1):.1f} %)", ""]
        if "--drop-trace" in sys.argv:
            os.remove(tpath)
    lines += ["| kernel | calls | total ms | avg us | % |", "|---|---:|---:|---:|---:|"]
    for r in stats[:40]:
        lines.append(f"| `{r['Name'][:110]}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:50]))


if __name__ == "__main__":
    main()
