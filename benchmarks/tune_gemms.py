"""Offline-tune the hipBLASLt / rocBLAS solutions of the decode-sized projections (PyTorch TunableOp)
and write them to django_assistant_bot_amd/tuning/ so every run uses the measured-fastest solution
instead of the library heuristic.  Tuning uses a rotating buffer (cold caches, like decode, which
streams 16 GB of weights per step).

    python benchmarks/tune_gemms.py [--model llama-3-8b] [--max-m 256] [--out PATH]

Prints cold timings of every shape before (heuristic) and after (tuned) as JSON lines.
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from django_assistant_bot_amd.models.configs import decoder_config  # noqa: E402
from django_assistant_bot_amd.engine.llm_engine import _bucket_sizes  # noqa: E402


def cold_time(M, N, K, iters=None):
    ncopy = max(2, int(2e9 // (N * K * 2)) + 1)
    ws = [torch.empty((N, K), dtype=torch.bfloat16, device="cuda").normal_(0, 0.02) for _ in range(ncopy)]
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    iters = iters or 2 * ncopy
    for i in range(3):
        F.linear(x, ws[i % ncopy])
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        F.linear(x, ws[i % ncopy])
    e.record()
    torch.cuda.synchronize()
    del ws
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--max-m", type=int, default=256)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--out", default=None)
    ap.add_argument("--prefill-m", default="", help="comma list of prefill chunk sizes to tune too")
    ap.add_argument("--no-decode", action="store_true")
    args = ap.parse_args()
    cfg = decoder_config(args.model)
    D, tp = cfg.head_dim, args.tp
    shapes = [((cfg.heads + 2 * cfg.kv_heads) * D // tp, cfg.hidden), (cfg.hidden, cfg.heads * D // tp),
              (2 * cfg.intermediate // tp, cfg.hidden), (cfg.hidden, cfg.intermediate // tp), (cfg.vocab_size, cfg.hidden)]
    arch = torch.cuda.get_device_properties(0).gcnArchName.split(":")[0]
    out = args.out or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                   "django_assistant_bot_amd", "tuning", f"tunableop_{args.model}_tp{tp}_{arch}.csv")
    buckets = [] if args.no_decode else _bucket_sizes(args.max_m)
    buckets += [int(m) for m in args.prefill_m.split(",") if m]
    before = {(M, N, K): cold_time(M, N, K, iters=10 if M > 4096 else None)
              for M in buckets for (N, K) in (shapes if M <= 4096 else shapes[:4])}

    import torch.cuda.tunable as tn
    tn.enable(True)
    tn.tuning_enable(True)
    if os.path.exists(out):
        tn.read_file(out)  # keep earlier results (decode) when adding prefill shapes
    tn.set_filename(out)
    tn.set_rotating_buffer_size(512)
    tn.set_max_tuning_duration(60)
    for M in buckets:
        for N, K in (shapes if M <= 4096 else shapes[:4]):
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
            F.linear(x, w)
            print(json.dumps({"tuned": [M, N, K]}), flush=True)
    torch.cuda.synchronize()
    # results are flushed to the file as they are tuned
    tn.tuning_enable(False)
    for (M, N, K), t0 in before.items():
        t1 = cold_time(M, N, K, iters=10 if M > 4096 else None)
        print(json.dumps({"M": M, "N": N, "K": K, "heuristic_us": round(t0, 1), "tuned_us": round(t1, 1),
                          "speedup": round(t0 / t1, 3)}), flush=True)
    print(json.dumps({"written": out}))


if __name__ == "__main__":
    main()
