"""The decode LM head (128,256 x 4096, batch 128) on every stream_gemm configuration that tiles it,
plain and grouped fragment layouts: cold weights (a rotation of copies > 2.5 GB), graph-timed, one
JSON line per (cfg, group) with us and TB/s.  Bit-equality of each grouped run to the plain one."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.kernel_bench import graph_time  # noqa: E402
from django_assistant_bot_amd import ops  # noqa: E402

M, N, K = 128, 128256, 4096


def main():
    nat = ops.native()
    x = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    cfgs = [c for c in (10, 14, 15, 21, 24, 26, 28, 29) if nat.stream_gemm_bn(c) and N % nat.stream_gemm_bn(c) == 0
            and nat.stream_gemm_max_m(c) >= M and nat.stream_gemm_shuffled(c)]
    for G in (1, 8):
        ws = [ops.shuffle_weights(w, G)] + [ops.shuffle_weights(torch.randn_like(w) * 0.02, G) for _ in range(2)]
        for cfg in cfgs:
            y = ops.stream_gemm(x, ws[0], cfg=cfg, nt=True, w_group=G)
            t = graph_time([lambda wk=wk: ops.stream_gemm(x, wk, cfg=cfg, nt=True, w_group=G) for wk in ws])
            print(json.dumps({"cfg": cfg, "bn": nat.stream_gemm_bn(cfg), "tiles": N // nat.stream_gemm_bn(cfg), "group": G,
                              "us": round(t * 1e6, 1), "tbps": round(N * K * 2 / t / 1e12, 2),
                              "checksum": float(y.float().sum())}), flush=True)
        del ws


if __name__ == "__main__":
    main()
