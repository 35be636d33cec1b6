"""Split-K choice for the decode projections, timed with their consumer: stream_gemm (M = 128,
cfg 10, nt) writing S fp32 slabs, then the slab RMSNorm (+ residual) that sums them -- the o and down
projections' pairs in the decode layer.  Weights rotate over copies larger than the MALL so every
launch streams from HBM; launches are captured in a HIP graph (as in the engine's decode step) and the replays timed as a
whole.  Prints one JSON line per (projection, splits)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from django_assistant_bot_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda")
    M, H = 128, 4096
    gain = torch.ones(H, device=dev, dtype=torch.bfloat16)
    res = (torch.randn(M, H, device=dev) * 0.5).to(torch.bfloat16)
    for name, K, splits in (("o", 4096, (2, 4, 8, 16)), ("down", 14336, (4, 8, 14, 16))):
        copies = max(2, (600 << 20) // (H * K * 2))
        ws = [ops.shuffle_weights((torch.randn(H, K, device=dev) * 0.02).to(torch.bfloat16)) for _ in range(copies)]
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        for s in splits:
            if K % (128 * s):
                continue

            def pair(i):
                slabs = ops.stream_gemm(x, ws[i % copies], splits=s, cfg=10, nt=True)
                return ops.rmsnorm(slabs, gain, 1e-5, residual=res)

            for i in range(2 * copies):
                pair(i)
            torch.cuda.synchronize()
            n = 8 * copies
            g = torch.cuda.CUDAGraph()  # captured like the engine's decode step: no host launch cost
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                pair(0)
                torch.cuda.synchronize()
                with torch.cuda.graph(g, stream=st):
                    for i in range(n):
                        pair(i)
            torch.cuda.current_stream().wait_stream(st)
            g.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                g.replay()
            b.record()
            torch.cuda.synchronize()
            n *= 5
            us = a.elapsed_time(b) * 1e3 / n
            print(json.dumps({"proj": name, "splits": s, "M": M, "N": H, "K": K, "pair_us": round(us, 2),
                              "weight_TBps": round(H * K * 2 / us / 1e6, 2)}), flush=True)
        del ws


if __name__ == "__main__":
    main()
