"""Decode projections at batch 128 on plain vs grouped fragment layouts (``shuffle_weights(w, G)``,
``stream_gemm(..., w_group=G)``): cold weights (a rotation of > 2.5 GB of copies), graph-timed, one
JSON line per projection with microseconds per call for G = 1 / 7 / 8.  Every grouped run is first
checked bit for bit against the plain layout's output (same math, different addressing)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.kernel_bench import graph_time  # noqa: E402
from django_assistant_bot_amd import ops  # noqa: E402

M = 128
SHAPES = (("gate_up", 28672, 4096, 20, 1, ops.EPI_SWIGLU8), ("gate_up", 28672, 4096, 22, 1, ops.EPI_SWIGLU8),
          ("gate_up", 28672, 4096, 41, 1, ops.EPI_SWIGLU8), ("gate_up", 28672, 4096, 42, 1, ops.EPI_SWIGLU8),
          ("qkv", 6144, 4096, 10, 4, ops.EPI_NONE),
          ("o", 4096, 4096, 10, 8, ops.EPI_NONE), ("down", 4096, 14336, 10, 8, ops.EPI_NONE))


def main():
    for name, N, K, cfg, S, epi in SHAPES:
        x = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
        ncopy = max(2, int(2.5e9 // (N * K * 2)) + 1)
        ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
        res = {"op": name, "M": M, "N": N, "K": K, "cfg": cfg, "S": S}
        kw = dict(splits=S, cfg=cfg, nt=True, epilogue=epi, slab_dtype=torch.bfloat16)
        base = None
        for G in (1, 7, 8) if cfg == 20 else (1, 8):
            if N % (16 * G):
                continue
            wl = [ops.shuffle_weights(w, G) for w in ws]
            y = ops.stream_gemm(x, wl[0], w_group=G, **kw)
            if base is None:
                base = y
            else:
                assert torch.equal(y, base), (name, G)
            res[f"g{G}_us"] = round(graph_time([lambda w=w: ops.stream_gemm(x, w, w_group=G, **kw) for w in wl]) * 1e6,
                                    1)
            del wl
        print(json.dumps(res), flush=True)
        del ws
    # prefill: the grouped gate_up copy through gemm_bt's dispatch (gemm_mid / gemm256), SwiGLU8
    N, K = 28672, 4096
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    plain, grp = ops.shuffle_weights(w), ops.shuffle_weights(w, 8)
    for Mp in (512, 2048, 8192, 32768):
        x = (torch.randn(Mp, K, device="cuda") * 0.5).to(torch.bfloat16)
        res = {"op": "gate_up_prefill", "M": Mp}
        y1 = ops.gemm_bt(x, plain, epilogue=ops.EPI_SWIGLU8, shuffled=True)
        assert torch.equal(ops.gemm_bt(x, grp, epilogue=ops.EPI_SWIGLU8, shuffled=True, b_group=8), y1), Mp
        for G, wk in ((1, plain), (8, grp)):
            t = graph_time([lambda: ops.gemm_bt(x, wk, epilogue=ops.EPI_SWIGLU8, shuffled=True, b_group=G)])
            res[f"g{G}_us"] = round(t * 1e6, 1)
            res[f"g{G}_tflops"] = round(2 * Mp * N * K / t / 1e12, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
