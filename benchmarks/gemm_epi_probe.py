"""What the gemm256 epilogue variants cost per shape: the same GEMM with no epilogue operands,
+bias, +bias+residual, +bias+GELU (bge-base encoder shapes at M = 65536 and Llama-3-8B prefill
shapes at M = 16384).  Graph-replayed back to back (weights rotated over copies larger than the
Infinity Cache are not needed here: these GEMMs are compute-bound).  One JSON line per arm.

    python benchmarks/gemm_epi_probe.py [bge|llama]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from django_assistant_bot_amd import ops  # noqa: E402


def graph_us(fn, reps=20):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = []
    for _ in range(5):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) * 1e3 / reps)
    return sorted(times)[len(times) // 2]


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    shapes = []
    if which in ("all", "bge"):
        M = 65536
        shapes += [("bge-qkv", M, 2304, 768), ("bge-o", M, 768, 768), ("bge-up", M, 3072, 768),
                   ("bge-down", M, 768, 3072)]
    if which in ("all", "llama"):
        M = 16384
        shapes += [("l8-qkv", M, 6144, 4096), ("l8-o", M, 4096, 4096), ("l8-down", M, 4096, 14336)]
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, M, N, K in shapes:
        a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        b = (torch.randn(N, K, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
        bias = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16)
        res = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        arms = {"plain": dict(), "bias": dict(bias=bias), "res": dict(residual=res),
                "bias_res": dict(bias=bias, residual=res), "bias_gelu": dict(bias=bias, epilogue=ops.EPI_GELU)}
        row = {"op": name, "M": M, "N": N, "K": K}
        for arm, kw in arms.items():
            us = graph_us(lambda: ops.kernels._gemm256_into(a, b, out, kw.get("bias"), kw.get("residual"),
                                                              kw.get("epilogue", ops.EPI_NONE), False))
            row[arm + "_us"] = round(us, 1)
            row[arm + "_tflops"] = round(2.0 * M * N * K / us / 1e6, 1)
        print(json.dumps(row), flush=True)
        del a, b, bias, res, out


if __name__ == "__main__":
    main()
