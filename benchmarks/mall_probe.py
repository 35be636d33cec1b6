"""Decode projection from HBM vs from the Infinity Cache (MALL): how much of the small decode GEMMs'
time is the cold weight stream?  The o (4096x4096) and qkv (6144x4096) projections run at 2.5-3 TB/s
in the decode layer (profiles/rocprof_r2_final.md), well under the gate_up / down streams.  This
times one stream_gemm launch (M = 128, the engine's cfg and split rule) after
  cold : a 2 GB temporal read that evicts the weights from L2 and MALL,
  warm : the same launch run just before (weights resident in MALL, 256 MB),
so the gap between the two bounds what a weight prefetch overlapped with the attention could save.
Prints one JSON line per (projection, arm)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from django_assistant_bot_amd import ops  # noqa: E402
from django_assistant_bot_amd.models.llama import LlamaModel  # noqa: E402


def main():
    dev = torch.device("cuda")
    flush = torch.empty(1 << 30, dtype=torch.bfloat16, device=dev).uniform_()
    M, K = 128, 4096
    x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    for name, N in (("o", 4096), ("qkv", 6144), ("down_k14336", 4096)):
        k = 14336 if name.startswith("down") else K
        xx = x if k == K else (torch.randn(M, k, device=dev) * 0.5).to(torch.bfloat16)
        w = (torch.randn(N, k, device=dev) * 0.02).to(torch.bfloat16)
        ws = ops.shuffle_weights(w)
        cfg = 10
        s = LlamaModel._stream_splits(N, k, ops.native().stream_gemm_bn(cfg))
        run = lambda nt: ops.stream_gemm(xx, ws, splits=s, cfg=cfg, nt=nt)  # noqa: E731
        for arm in ("cold", "warm_nt", "warm_temporal"):
            ts = []
            for _ in range(30):
                if arm == "cold":
                    flush.sum()
                else:
                    run(arm == "warm_nt")
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                run(True)
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            ts.sort()
            med = ts[len(ts) // 2]
            print(json.dumps({"proj": name, "arm": arm, "M": M, "N": N, "K": k, "splits": s, "cfg": cfg,
                              "median_us": round(med, 2), "min_us": round(ts[0], 2),
                              "TBps": round(N * k * 2 / med / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
