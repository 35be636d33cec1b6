"""Where a gemm256 tile's time goes: per-tile s_memtime stamps (diagnostic STAMP instantiation of
gemm256.hip) on short-K (bge, index-search) and long-K (Llama prefill) shapes.

For every workgroup and tile, wave 0 records the clock at the tile's first K-iteration, the cycles
of its K-loop and of its epilogue.  Reported per shape (medians over workgroups and tiles, shader
clock cycles): K-loop cycles per tile and per 64-deep K-tile, epilogue cycles, the transition
between one tile's epilogue end and the next tile's start, and the first tile's K-loop (which
includes the workgroup's prologue wait).  The stamps cost wave 0 one vector store per tile.

    python benchmarks/gemm_stamps.py [--shapes bge-qkv,llama-o] [--cand 0.0016 0.0004]

--cand runs the index search's candidate GEMM (thresholds set for the given hit fraction) instead
of / besides the plain shapes; its epilogue cycles include the candidate-list flushes.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from django_assistant_bot_amd import ops  # noqa: E402
from django_assistant_bot_amd.ops.kernels import native, ptr, stream  # noqa: E402

SHAPES = {
    "bge-qkv": (65536, 2304, 768, "bias", False),
    "bge-o": (65536, 768, 768, "bias+res", False),
    "bge-up": (65536, 3072, 768, "gelu", False),
    "bge-down": (65536, 768, 3072, "bias+res", False),
    "cand-shape": (512, 262144, 768, "none", True),  # the index search's GEMM shape (plain epilogue)
    "llama-qkv": (32768, 6144, 4096, "none", True),
    "llama-o": (32768, 4096, 4096, "res", True),
}


def rand(shape, scale=1.0):
    return ((torch.rand(shape, device="cuda") * 2 - 1) * scale).to(torch.bfloat16)


def run(name, M, N, K, kind, shuf, reps, aux=0):
    a, w = rand((M, K)), rand((N, K), 0.05)
    wb = ops.shuffle_weights(w) if shuf else w
    c = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
    bias = rand((N,), 0.5) if "bias" in kind or kind == "gelu" else None
    res = rand((M, N)) if "res" in kind else None
    tiles = (M + 255) // 256 * (N // 256)
    per_wg = -(-tiles // 256) + 1
    st = torch.zeros((256, per_wg, 4), dtype=torch.int32, device="cuda")
    epi = 1 if kind == "gelu" else 0
    nat = native()
    out = []
    for _ in range(reps):
        st.zero_()
        grid = nat.gemm256_stamped(ptr(a), K, ptr(wb), ptr(c), ptr(bias), ptr(res), M, N, K, epi, int(shuf), ptr(st),
                                   per_wg, stream(a), aux)
        torch.cuda.synchronize()
        out.append(st[:grid].cpu().numpy().astype(np.uint32))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(10):
        nat.gemm256_stamped(ptr(a), K, ptr(wb), ptr(c), ptr(bias), ptr(res), M, N, K, epi, int(shuf), ptr(st), per_wg,
                            stream(a), aux)
    ev[1].record()
    torch.cuda.synchronize()
    res = {"shape": name, "M": M, "N": N, "K": K, "epilogue": kind, "store_aux": aux,
           "us": round(ev[0].elapsed_time(ev[1]) * 100.0, 1)}
    res.update(summarize(out[-1], K, tiles))
    return res


def run_cand(M, N, K, hit_frac, reps):
    """The index search's candidate GEMM (shuffled index copy, thresholds from a 64k-row slice at the
    given hit fraction: 0.0016 = the 1/64 sample's k = 250 bound over 10M rows)."""
    a, w = rand((M, K)), rand((N, K))
    a = a / a.float().norm(dim=1, keepdim=True).to(a.dtype)
    w = w / w.float().norm(dim=1, keepdim=True).to(w.dtype)
    wb = ops.shuffle_weights(w)
    del w
    sl = rand((65536, K)).float()
    sc = a.float() @ (sl / sl.norm(dim=1, keepdim=True)).T
    kk = max(1, int(round(65536 * hit_frac)))
    thr = sc.topk(kk, dim=1).values[:, -1].contiguous()
    del sc, sl
    cap = max(64, int(N * hit_frac * 4))
    cnt = torch.zeros(M, dtype=torch.int32, device="cuda")
    cv = torch.empty(M * cap, dtype=torch.float32, device="cuda")
    ci = torch.empty(M * cap, dtype=torch.int32, device="cuda")
    tiles = (M + 255) // 256 * ((N + 255) // 256)
    per_wg = -(-tiles // 256) + 1
    st = torch.zeros((256, per_wg, 4), dtype=torch.int32, device="cuda")
    nat = native()

    def launch():
        cnt.zero_()
        return nat.gemm256_candidates_stamped(ptr(a), K, ptr(wb), M, N, K, wb.shape[0], ptr(thr), ptr(cnt), ptr(cv),
                                              ptr(ci), cap, ptr(st), per_wg, stream(a))
    out = []
    for _ in range(reps):
        st.zero_()
        grid = launch()
        torch.cuda.synchronize()
        out.append(st[:grid].cpu().numpy().astype(np.uint32))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(10):
        launch()
    ev[1].record()
    torch.cuda.synchronize()
    res = summarize(out[-1], K, tiles)
    res.update({"shape": "cand", "M": M, "N": N, "K": K, "hit_frac": hit_frac,
                "hits_per_tile": round(float(cnt.sum()) / tiles, 1), "us": round(ev[0].elapsed_time(ev[1]) * 100.0, 1)})
    return res


def summarize(s, K, tiles):
    t0 = s[:, :, 0].astype(np.uint64) | (s[:, :, 1].astype(np.uint64) << np.uint64(32))
    loop, epi_c = s[:, :, 2].astype(np.int64), s[:, :, 3].astype(np.int64)
    valid = t0 > 0
    first = loop[:, 0][valid[:, 0]]
    later = loop[:, 1:][valid[:, 1:]]
    trans = []
    for g in range(s.shape[0]):
        n = int(valid[g].sum())
        for i in range(n - 1):
            trans.append(int(t0[g, i + 1]) - int(t0[g, i]) - int(loop[g, i]) - int(epi_c[g, i]))
    span = [int(t0[g, int(valid[g].sum()) - 1]) + int(loop[g, int(valid[g].sum()) - 1]) +
            int(epi_c[g, int(valid[g].sum()) - 1]) - int(t0[g, 0]) for g in range(s.shape[0]) if valid[g, 0]]
    kt = K // 64
    ev = epi_c[valid]
    return {"tiles_per_wg": round(tiles / s.shape[0], 2),
            "loop_cyc_median": int(np.median(later)) if later.size else None,
            "loop_cyc_per_ktile": round(float(np.median(later)) / kt, 1) if later.size else None,
            "first_tile_loop_cyc": int(np.median(first)),
            "epilogue_cyc_median": int(np.median(ev)), "epilogue_cyc_mean": int(np.mean(ev)),
            "epilogue_cyc_p95": int(np.percentile(ev, 95)),
            "transition_cyc_median": int(np.median(trans)) if trans else None,
            "wg_span_cyc_median": int(np.median(span)),
            "loop_share": round(float(loop[valid].sum()) / float(np.sum(span)), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--aux", type=int, nargs="+", default=[0],
                    help="epilogue store cache policies to compare (0, 2 = nt, 16 = sc1, 18 = sc1 + nt)")
    ap.add_argument("--cand", type=float, nargs="*", default=[],
                    help="hit fractions for the candidate-GEMM stamps (0.0016 = the 1/64 sample's bound)")
    ap.add_argument("--cand-m", type=int, default=512)
    ap.add_argument("--cand-n", type=int, default=1 << 20)
    args = ap.parse_args()
    torch.manual_seed(0)
    for frac in args.cand:
        print(json.dumps(run_cand(args.cand_m, args.cand_n, 768, frac, args.reps)), flush=True)
        torch.cuda.empty_cache()
    for name in (args.shapes.split(",") if args.shapes else []):
        for aux in args.aux:
            print(json.dumps(run(name, *SHAPES[name], args.reps, aux)), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
