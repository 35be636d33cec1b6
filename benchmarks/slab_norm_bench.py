"""Graph-timed split-K slab RMSNorm at the Llama-3-8B decode shape (S fp32 slabs of 128 x 4096 +
residual; S = 8 is the o / down split, S = 4 has the bytes 8 bf16 slabs would have; S = 1 is a plain
bf16-sized read of one fp32 tensor): 64 launches per replay, microseconds per call."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from django_assistant_bot_amd import ops  # noqa: E402

M, N = 128, 4096
w = (torch.randn(N, device="cuda")).to(torch.bfloat16)
r = (torch.randn(M, N, device="cuda")).to(torch.bfloat16)
for S in (8, 4, 2):
    slabs = [torch.randn(S, M, N, device="cuda") for _ in range(8)]
    for _ in range(3):
        ops.rmsnorm(slabs[0], w, 1e-5, residual=r)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for i in range(64):
                ops.rmsnorm(slabs[i % 8], w, 1e-5, residual=r)
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"op": f"rmsnorm-slab{S}-{M}x{N}", "us": round(e0.elapsed_time(e1) * 1000 / (20 * 64), 2)}),
          flush=True)
    del g, slabs
