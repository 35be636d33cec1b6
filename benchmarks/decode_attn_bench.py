"""Paged decode attention at the headline decode shape: 128 sequences with mixed context lengths
(the bench's ~1.0-1.5k tokens), Llama-3-8B heads (32 q / 8 kv, D 128), block size 64, shuffled block
tables.  Compares dispatch orders (batch order vs longest-first) and partition sizes; uniform
contexts of the same mean give the no-imbalance reference.  Graph-timed: N launches captured in one
HIP graph, replayed; K/V rotate over several copies so the 650 MB working set stays cold as in the
model (where 16 GB of weights stream between two layers' attention).

    python benchmarks/decode_attn_bench.py [--batch 128] [--copies 3]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from django_assistant_bot_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--copies", type=int, default=3)
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--pool-blocks", type=int, default=0,
                    help="cache blocks per copy (0: exactly the live ones); a pool the size of the "
                         "engine's (~24k blocks = 3 GB per layer's K) spreads the live blocks over it")
    ap.add_argument("--between", type=int, default=0,
                    help="stream a gate_up-sized decode GEMM (235 MB of weights, cold copies) between "
                         "attention launches, as the layer does (0: attention back to back)")
    ap.add_argument("--between-rows", type=int, default=28672, help="weight rows of that GEMM (K 4096)")
    ap.add_argument("--between-kind", choices=("gemm", "copy", "spin"), default="gemm",
                    help="what runs between attention launches: the streaming GEMM, a device copy of "
                         "the same bytes (HBM traffic without MFMA), or a spin kernel of about the "
                         "same duration (no memory traffic)")
    ap.add_argument("--parts", default="2048,1024,512", help="partition sizes to time")
    ap.add_argument("--dists", default="mixed,uniform", help="context distributions to time")
    ap.add_argument("--spread", choices=("random", "compact"), default="random",
                    help="live blocks drawn at random from the pool, or the lowest ids in order")
    a = ap.parse_args()
    Hq, Hkv, D, bs, B = 32, 8, 128, 64, a.batch
    g = torch.Generator().manual_seed(0)
    for dist_name in a.dists.split(","):
        if dist_name == "mixed":
            ctx_h = torch.randint(950, 1450, (B,), generator=g)
        else:
            ctx_h = torch.full((B,), 1200)
        nbs = [math.ceil(int(c) / bs) for c in ctx_h]
        nb = sum(nbs)
        pool = max(nb, a.pool_blocks)
        caches = []
        for _ in range(a.copies):
            kc = torch.empty(pool, Hkv, bs, D, device="cuda", dtype=torch.bfloat16).normal_()
            caches.append((kc, torch.empty_like(kc).normal_()))
        perm = torch.randperm(pool, generator=g)[:nb] if a.spread == "random" else torch.arange(nb)
        bt = torch.zeros((B, max(nbs)), dtype=torch.int32)
        o = 0
        for i, n in enumerate(nbs):
            bt[i, :n] = perm[o:o + n].to(torch.int32)
            o += n
        bt = bt.cuda()
        ctx = ctx_h.to(torch.int32).cuda()
        q = torch.randn(B, Hq, D, device="cuda").to(torch.bfloat16)
        longest = torch.argsort(ctx_h, descending=True).to(torch.int32).cuda()
        byts = 2.0 * float(ctx_h.sum()) * Hkv * D * 2
        res = {"op": "paged-decode", "ctx": dist_name, "B": B, "mean_ctx": int(ctx_h.float().mean()),
               "GB": round(byts / 1e9, 3), "pool_blocks": pool, "spread": a.spread}
        ref = None
        gemm_w = [ops.shuffle_weights(torch.randn(a.between_rows, 4096, device="cuda").to(torch.bfloat16))
                  for _ in range(2)] if a.between else []
        gemm_x = torch.randn(B, 4096, device="cuda").to(torch.bfloat16)
        copy_dst = torch.empty_like(gemm_w[0]) if a.between and a.between_kind == "copy" else None

        def between(i):
            if a.between_kind == "gemm":
                ops.stream_gemm(gemm_x, gemm_w[i % 2], cfg=10, nt=os.environ.get("BETWEEN_NT", "1") == "1")
            elif a.between_kind == "copy":
                copy_dst.copy_(gemm_w[i % 2])
            else:
                torch.cuda._sleep(100_000)  # ~50 us of spinning at ~2 GHz, no memory traffic

        for part in (int(x) for x in a.parts.split(",")):
            ws = ops.DecodeWorkspace(B, Hq, D, math.ceil(4096 / part), "cuda")
            for oname, order in (("batch", None), ("longest", longest)):
                outs = []

                def run():
                    for i, (kc, vc) in enumerate(caches):
                        if gemm_w:
                            between(i)
                        outs.append(ops.paged_decode(q, kc, vc, bt, ctx, part, ws, order=order))
                run()
                torch.cuda.synchronize()
                if ref is None:
                    ref = outs[0].float()
                err = (outs[0].float() - ref).abs().max().item()
                outs.clear()
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    for _ in range(a.iters):
                        run()
                torch.cuda.synchronize()
                graph.replay()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                graph.replay()
                e.record()
                torch.cuda.synchronize()
                t = s.elapsed_time(e) / 1e3 / (a.iters * a.copies)
                res[f"p{part}_{oname}_us"] = round(t * 1e6, 1)
                res[f"p{part}_{oname}_tbps"] = round(byts / t / 1e12, 2)
                res[f"p{part}_{oname}_err"] = round(err, 4)
                del graph, outs
        print(json.dumps(res), flush=True)
        del caches


if __name__ == "__main__":
    main()
