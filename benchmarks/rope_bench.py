"""Graph-timed decode RoPE + KV-cache write at the Llama-3-8B decode shape (4 fp32 split-K slabs of
the QKV projection, 128 tokens): 64 launches per replay, microseconds per call."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from django_assistant_bot_amd import ops  # noqa: E402
from django_assistant_bot_amd.ops import reference as ref  # noqa: E402

S, T, Hq, Hkv, D, bs = 4, 128, 32, 8, 128, 64
slabs = [torch.randn(S, T, (Hq + 2 * Hkv) * D, device="cuda") for _ in range(4)]
cs = ref.rope_cos_sin(ref.llama3_inv_freq(D, 500000.0, {"factor": 8.0}), 4096).to("cuda")
pos = torch.randint(0, 4000, (T,), device="cuda", dtype=torch.int32)
nb = 4096
kc = torch.zeros(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
vc = torch.zeros_like(kc)
slots = torch.randperm(nb * bs, device="cuda")[:T].to(torch.int64)
for _ in range(3):
    ops.rope_kv_write(slabs[0], pos, cs, kc, vc, slots, Hq, Hkv, D)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(st):
    with torch.cuda.graph(g, stream=st):
        for i in range(64):
            ops.rope_kv_write(slabs[i % 4], pos, cs, kc, vc, slots, Hq, Hkv, D)
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
print(json.dumps({"op": "rope-kv-slab4-128tok", "us": round(e0.elapsed_time(e1) * 1000 / (20 * 64), 2)}))
