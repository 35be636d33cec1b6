"""Paged-decode sweep: time vs (max_parts, part_size) at fixed batch/context (diagnostic)."""
import math, os, sys, json
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from django_assistant_bot_amd import ops
from benchmarks.kernel_bench import timeit

B, Hq, Hkv, D, bs = 64, 32, 8, 128, 64
for C in (1300, 4000):
    nb = B * math.ceil(C / bs)
    kc = torch.randn(nb, Hkv, bs, D, device="cuda").to(torch.bfloat16); vc = torch.randn_like(kc)
    bt = torch.arange(nb, dtype=torch.int32, device="cuda").view(B, -1)
    q = torch.randn(B, Hq, D, device="cuda").to(torch.bfloat16)
    ctx = torch.full((B,), C, dtype=torch.int32, device="cuda")
    for ps in (256, 512, 1024):
        for mp in (math.ceil(C / ps), 8, 16, 32):
            if mp * ps < C: continue
            ws = ops.DecodeWorkspace(B, Hq, D, mp, "cuda")
            t = timeit(lambda: ops.paged_decode(q, kc, vc, bt, ctx, ps, ws), iters=30)
            print(json.dumps({"ctx": C, "part_size": ps, "max_parts": mp, "us": round(t * 1e6, 1),
                              "gbps": round(2.0 * B * C * Hkv * D * 2 / t / 1e9)}), flush=True)
