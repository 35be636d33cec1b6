"""Small prefill steps (a few hundred tokens: single interactive prompts, the tail step of a batch):
each Llama-3-8B projection through gemm_bt's MFMA dispatch against the streaming decode kernel
(stream_gemm at the decoder's own cfg / K-split choice, slabs summed by slab_reduce where a consumer
would sum them), cold weights, graph-timed, us."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.kernel_bench import graph_time  # noqa: E402
from django_assistant_bot_amd import ops  # noqa: E402
from django_assistant_bot_amd.models.llama import LlamaModel  # noqa: E402

SHAPES = (("qkv", 6144, 4096, ops.EPI_NONE), ("o", 4096, 4096, ops.EPI_NONE),
          ("gate_up", 28672, 4096, ops.EPI_SWIGLU8), ("down", 4096, 14336, ops.EPI_NONE))


def main():
    m = LlamaModel.__new__(LlamaModel)  # only the stream-choice helpers (no weights)
    for name, N, K, epi in SHAPES:
        G = LlamaModel.PROJ_GROUPS.get(name, 1)
        ws = [ops.shuffle_weights((torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16), G)
              for _ in range(max(2, int(2.5e9 // (N * K * 2)) + 1))]
        for M in (32, 64, 128, 129, 160, 187, 224, 256):
            x = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
            res = {"op": name, "M": M}
            t = graph_time([lambda w=w: ops.gemm_bt(x, w, epilogue=epi, shuffled=True, b_group=G) for w in ws])
            res["gemm_bt_us"] = round(t * 1e6, 1)
            if ops.kernels.gemm_mid_ok(M, N, K, K):
                t = graph_time([lambda w=w: ops.kernels.gemm_mid(x, w, epilogue=epi, b_group=G) for w in ws])
                res["gemm_mid_us"] = round(t * 1e6, 1)
            cfg, s = m._stream_choice(name, M, N, K)
            if cfg >= 0:
                if epi != ops.EPI_NONE or s == 1:
                    f = lambda w: ops.stream_gemm(x, w, epilogue=epi, nt=True, cfg=cfg, w_group=G)  # noqa: E731
                else:
                    f = lambda w: ops.slab_reduce(ops.stream_gemm(x, w, splits=s, cfg=cfg, nt=True,  # noqa: E731
                                                                  slab_dtype=torch.bfloat16, w_group=G))
                t = graph_time([lambda w=w: f(w) for w in ws])
                res.update(stream_cfg=cfg, splits=s, stream_us=round(t * 1e6, 1))
            print(json.dumps(res), flush=True)
        del ws


if __name__ == "__main__":
    main()
