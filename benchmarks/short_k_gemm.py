"""The encoder's GEMMs (bge-base, 262,144-token batch: K = 768 / 3072) on the phased 256 x 256 kernel
(gemm256, the dispatch from M = 1024) against gemm.hip's own tiling (128 x 128 / 256 x 256 with several
workgroups per CU, so one tile's epilogue overlaps another's K loop), row-major weights with bias /
GELU / residual as the encoder runs them; graph-timed, us and TF/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.kernel_bench import graph_time  # noqa: E402
from django_assistant_bot_amd import ops  # noqa: E402
from django_assistant_bot_amd.ops.kernels import native, ptr, stream  # noqa: E402

M = 262144
SHAPES = (("qkv", 2304, 768, ops.EPI_NONE, False), ("o", 768, 768, ops.EPI_NONE, True),
          ("up", 3072, 768, ops.EPI_GELU, False), ("down", 768, 3072, ops.EPI_NONE, True))


def main():
    for name, N, K, epi, res in SHAPES:
        A = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
        B = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
        bias = torch.randn(N, device="cuda").to(torch.bfloat16)
        r = torch.randn(M, N, device="cuda").to(torch.bfloat16) if res else None
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)

        def g256():
            ops.kernels._gemm256_into(A, B, out, bias, r, epi, False)

        def gbt():
            native().gemm_bt(ptr(A), K, ptr(B), K, ptr(out), N, ptr(bias), ptr(r), N if res else 0, M, N, K, int(epi),
                             0, 0, 0, 0, 0, stream(A), 0, 1)

        g256()
        ref = out.clone()
        gbt()
        diff = float((out.float() - ref.float()).abs().max())
        t1, t2 = graph_time([g256]), graph_time([gbt])
        fl = 2.0 * M * N * K
        print(json.dumps({"op": name, "N": N, "K": K, "gemm256_us": round(t1 * 1e6, 1), "gemm_bt_us": round(t2 * 1e6, 1),
                          "gemm256_tflops": round(fl / t1 / 1e12), "gemm_bt_tflops": round(fl / t2 / 1e12),
                          "max_diff": diff}), flush=True)


if __name__ == "__main__":
    main()
