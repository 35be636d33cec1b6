"""Per-kernel timings on the real model shapes (bf16, random data).

GEMM: native MFMA ``gemm_bt`` (row-major B) vs hipBLASLt (torch.nn.functional.linear) on the Llama-3-8B decode /
prefill and bge-base encoder projections; attention: flash prefill, paged decode; selection kernels.
Prints one JSON line per measurement (TFLOP/s and effective GB/s).
"""
import json
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from django_assistant_bot_amd import ops  # noqa: E402


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3


def emit(**kw):
    print(json.dumps(kw), flush=True)


def gemm_suite(which):
    shapes = []
    for M in (1, 32, 64, 128, 256):
        shapes += [("llama8b-qkv", M, 6144, 4096), ("llama8b-o", M, 4096, 4096), ("llama8b-gateup", M, 28672, 4096),
                   ("llama8b-down", M, 4096, 14336)]
    shapes += [("llama8b-lmhead", 64, 128256, 4096)]
    for M in (4096, 16384):
        shapes += [("llama8b-qkv", M, 6144, 4096), ("llama8b-gateup", M, 28672, 4096), ("llama8b-down", M, 4096, 14336)]
    for M in (2048, 32768, 65536):
        shapes += [("bge-qkv", M, 2304, 768), ("bge-o", M, 768, 768), ("bge-up", M, 3072, 768), ("bge-down", M, 768, 3072)]
    shapes += [("index-scan", 64, 1_000_000, 768), ("index-scan", 512, 1_000_000, 768)]
    for name, M, N, K in shapes:
        if which and which not in name:
            continue
        a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        b = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
        flop = 2.0 * M * N * K
        byts = 2.0 * (M * K + N * K + M * N)
        res = {"op": name, "M": M, "N": N, "K": K}
        if name == "index-scan":
            t_nat = timeit(lambda: ops.gemm_bt(a, b, epilogue=ops.EPI_SCORES, out_f32=True), iters=5)
            t_lib = timeit(lambda: torch.mm(a, b.t()).float(), iters=5)
            byts = 2.0 * (M * K + N * K) + 4.0 * M * N
        else:
            t_nat = timeit(lambda: ops.gemm_bt(a, b))
            t_lib = timeit(lambda: F.linear(a, b))
        res.update(native_us=round(t_nat * 1e6, 1), hipblaslt_us=round(t_lib * 1e6, 1),
                   native_tflops=round(flop / t_nat / 1e12, 1), hipblaslt_tflops=round(flop / t_lib / 1e12, 1),
                   native_gbps=round(byts / t_nat / 1e9), hipblaslt_gbps=round(byts / t_lib / 1e9))
        emit(**res)
        del a, b


def graph_time(calls, reps=5):
    """Device time per call of a list of zero-arg launches, captured into one HIP graph and replayed
    (no host launch overhead in the number: the decode step replays a graph too)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for f in calls:
            f()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for f in calls:
            f()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 1e3 / len(calls))
    del g
    return best


def stream_sweep(which, Ms=(128,)):
    """Decode projections of Llama-3-8B (+ LM head) at decode batch M with cold weights (a rotation
    of > 2 GB of weight copies, as in a decode step that streams 16 GB): hipBLASLt vs the
    warp-specialised stream kernel per configuration and split count.  Graph-
    timed, microseconds per call."""
    shapes = (("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
              ("lm_head", 128256, 4096))
    n_cfg = 20
    cfgs = [int(c) for c in os.environ.get("STREAM_CFGS", "").split(",") if c] or list(range(n_cfg))
    for M in Ms:
        for name, N, K in shapes:
            if which and which not in name:
                continue
            a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            # STREAM_WARM=1: one copy, replayed back to back (weights served from the Infinity Cache
            # when they fit in its 256 MB: bounds what a prefetch of the next GEMM's weights could buy)
            ncopy = 1 if os.environ.get("STREAM_WARM") else max(2, int(2.5e9 // (N * K * 2)) + 1)
            ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
            res = {"op": name, "M": M, "N": N, "K": K, "weights_mb": round(N * K * 2 / 1e6, 1)}
            res["hipblaslt_us"] = round(graph_time([lambda w=w: F.linear(a, w) for w in ws]) * 1e6, 1)
            for cfg in cfgs:
                bn, mm = ops.native().stream_gemm_bn(cfg), ops.native().stream_gemm_max_m(cfg)
                if M > mm or N % bn:
                    continue
                wl = ws if not ops.native().stream_gemm_shuffled(cfg) else [ops.shuffle_weights(w) for w in ws]
                for S in (1, 2, 4, 8):
                    if K % (S * 128) or (N // bn) * S > 2048 or (N // bn) * S < 96:
                        continue
                    slabs = torch.empty((S, M, N), dtype=torch.float32, device="cuda") if S > 1 else None
                    for nt in ((0, 1) if os.environ.get("STREAM_NT") else (0,)):
                        t = graph_time([lambda w=w: ops.stream_gemm(a, w, splits=S, out=slabs, nt=nt, cfg=cfg)
                                        for w in wl])
                        res[f"c{cfg}_S{S}{'nt' if nt else ''}_us"] = round(t * 1e6, 1)
            best = min((v, k) for k, v in res.items() if k.endswith("_us"))
            res["best"] = best[1]
            res["best_tbps"] = round(N * K * 2 / best[0] / 1e12, 2)
            emit(**res)
            del ws


def attn_suite():
    # prefill: 16 sequences x 1024 tokens, Llama-3-8B heads
    B, T, Hq, Hkv, D, bs = 16, 1024, 32, 8, 128, 64
    nb = B * T // bs
    kc = torch.randn(nb, Hkv, bs, D, device="cuda").to(torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.arange(nb, dtype=torch.int32, device="cuda").view(B, T // bs)
    q = torch.randn(B * T, Hq, D, device="cuda").to(torch.bfloat16)
    cu = torch.arange(0, B * T + 1, T, dtype=torch.int32, device="cuda")
    ctx = torch.full((B,), T, dtype=torch.int32, device="cuda")
    t = timeit(lambda: ops.flash_attention_paged(q, kc, vc, bt, cu, ctx, T, causal=True))
    flop = 4.0 * B * Hq * T * T * D / 2
    emit(op="flash-prefill-causal", B=B, T=T, us=round(t * 1e6, 1), tflops=round(flop / t / 1e12, 1))
    # A/B of the software-pipelined V reads (DAB_FLASH_VPIPE), interleaved rounds in this process
    # A/B of the kernel variants (env-selected per launch), interleaved rounds in this process:
    # base = unpipelined V reads, vpipe = pipelined (default), w8 = 8 waves + 3-deep K/V ring,
    # pair = (long, short) causal query-block pairs, G per workgroup (default: G from the launch
    # size; pair-g1 / pair-g4 force G)
    arms = {"base": {"DAB_FLASH_VPIPE": "0"}, "vpipe": {"DAB_FLASH_PAIR": "0"}, "pair": {},
            "pair-g1": {"DAB_FLASH_G": "1"}, "pair-g4": {"DAB_FLASH_G": "4"}, "pair-1bar": {"DAB_FLASH_1BAR": "1"}, "pair-sms": {"DAB_FLASH_SMS": "1"},
            "pair-sgb": {"DAB_FLASH_SGB": "1"},
            "q64": {"DAB_FLASH_Q64": "1"}, "w8": {"DAB_FLASH_W8": "1"}}
    if os.environ.get("ATTN_ARMS"):  # e.g. ATTN_ARMS=vpipe,pair (a short run for PMC passes)
        arms = {a: arms[a] for a in os.environ["ATTN_ARMS"].split(",")}

    def with_env(env, fn):
        old = {k: os.environ.get(k) for k in ("DAB_FLASH_VPIPE", "DAB_FLASH_W8", "DAB_FLASH_PAIR", "DAB_FLASH_G",
                                           "DAB_FLASH_1BAR", "DAB_FLASH_Q64", "DAB_FLASH_SMS",
                                           "DAB_FLASH_SGB")}
        for k in old:
            os.environ.pop(k, None)
        os.environ.update(env)
        try:
            return fn()
        finally:
            for k, v in old.items():
                os.environ.pop(k, None)
                if v is not None:
                    os.environ[k] = v

    for causal in (True, False):
        run = lambda: ops.flash_attention_paged(q, kc, vc, bt, cu, ctx, T, causal=causal)  # noqa: E731
        ref_out = with_env({"DAB_FLASH_VPIPE": "0"}, run)
        ab = {a: [] for a in arms}
        for _ in range(5):
            for arm, env in arms.items():
                ab[arm].append(with_env(env, lambda: timeit(run)))
        fl = flop if causal else 2 * flop
        for arm, ts in ab.items():
            err = (with_env(arms[arm], run).float() - ref_out.float()).abs().max()
            tm = sorted(ts)[len(ts) // 2]
            emit(op=f"flash-prefill-{'causal' if causal else 'full'}-{arm}", B=B, T=T, us=round(tm * 1e6, 1),
                 tflops=round(fl / tm / 1e12, 1), max_diff_vs_base=round(float(err), 5))
    # the model's prefill form: q read from the qkv projection (row stride (Hq + 2 Hkv) D), without
    # and with RoPE applied on load
    qkv = torch.randn(B * T, (Hq + 2 * Hkv) * D, device="cuda").to(torch.bfloat16)
    qs = qkv[:, :Hq * D].view(B * T, Hq, D)
    pos = torch.arange(T, dtype=torch.int32, device="cuda").repeat(B)
    cs = ops.reference.rope_cos_sin(ops.reference.llama3_inv_freq(D, 500000.0, None), 8192).cuda()
    t = timeit(lambda: ops.flash_attention_paged(qs, kc, vc, bt, cu, ctx, T, causal=True))
    emit(op="flash-prefill-causal-qkv-strided", B=B, T=T, us=round(t * 1e6, 1), tflops=round(flop / t / 1e12, 1))
    t = timeit(lambda: ops.flash_attention_paged(qs, kc, vc, bt, cu, ctx, T, causal=True, rope=(pos, cs)))
    emit(op="flash-prefill-causal-rope", B=B, T=T, us=round(t * 1e6, 1), tflops=round(flop / t / 1e12, 1))
    # encoder: 256 x 128 tokens, bge-base heads (packed)
    B2, T2, H2, D2 = 256, 128, 12, 64
    qkv = torch.randn(B2 * T2, 3 * H2 * D2, device="cuda").to(torch.bfloat16)
    cu2 = torch.arange(0, B2 * T2 + 1, T2, dtype=torch.int32, device="cuda")
    qv = qkv[:, :H2 * D2].view(-1, H2, D2)
    kv = qkv[:, H2 * D2:2 * H2 * D2].view(-1, H2, D2)
    vv = qkv[:, 2 * H2 * D2:].view(-1, H2, D2)
    t = timeit(lambda: ops.flash_attention_packed(qv, kv, vv, cu2, cu2, T2))
    flop = 4.0 * B2 * H2 * T2 * T2 * D2
    emit(op="flash-encoder", B=B2, T=T2, us=round(t * 1e6, 1), tflops=round(flop / t / 1e12, 1))
    # the embed bench's shape: one 262,144-token packed batch of 25-75-token chunks (mean ~50), in
    # length order as the engine packs them; A/B of the 5-waves-per-SIMD variant (DAB_ENC_W5)
    g = torch.Generator().manual_seed(0)
    lens = torch.sort(torch.randint(25, 76, (5300,), generator=g), descending=True).values
    lens = lens[torch.cumsum(lens, 0) <= 262144]
    cu3 = torch.zeros(len(lens) + 1, dtype=torch.int32)
    cu3[1:] = torch.cumsum(lens, 0)
    cu3 = cu3.cuda()
    T3 = int(cu3[-1])
    qkv3 = torch.randn(T3, 3 * H2 * D2, device="cuda").to(torch.bfloat16)
    q3, k3, v3 = (qkv3[:, i * H2 * D2:(i + 1) * H2 * D2].view(-1, H2, D2) for i in range(3))
    mx3 = int(lens.max())
    run3 = lambda: ops.flash_attention_packed(q3, k3, v3, cu3, cu3, mx3)  # noqa: E731
    env3 = {"base": {"DAB_ENC_W5": "0"}, "w5": {}, "persist": {"DAB_ENC_PERSIST": "1"}}

    def with_env3(env, fn):
        for k in ("DAB_ENC_W5", "DAB_ENC_PERSIST"):
            os.environ.pop(k, None)
        os.environ.update(env)
        try:
            return fn()
        finally:
            for k in ("DAB_ENC_W5", "DAB_ENC_PERSIST"):
                os.environ.pop(k, None)

    ref3 = with_env3(env3["base"], run3)
    res3 = {a: [] for a in env3}
    for _ in range(5):
        for arm, env in env3.items():
            res3[arm].append(with_env3(env, lambda: timeit(run3)))
    byts3 = T3 * 4 * H2 * D2 * 2  # q, k, v read + o written
    for arm, ts in res3.items():
        err3 = (with_env3(env3[arm], run3).float() - ref3.float()).abs().max()
        tm = sorted(ts)[len(ts) // 2]
        emit(op=f"flash-encoder-embedbatch-{arm}", tokens=T3, seqs=len(lens), us=round(tm * 1e6, 1),
             tbps=round(byts3 / tm / 1e12, 2), max_diff_vs_base=round(float(err3), 5))
    # decode: 64 sequences x 1300 context
    for Bd, C in ((64, 1300), (256, 1300), (64, 4000)):
        nbd = Bd * math.ceil(C / bs)
        kc = torch.randn(nbd, Hkv, bs, D, device="cuda").to(torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = torch.arange(nbd, dtype=torch.int32, device="cuda").view(Bd, -1)
        qd = torch.randn(Bd, Hq, D, device="cuda").to(torch.bfloat16)
        ctx = torch.full((Bd,), C, dtype=torch.int32, device="cuda")
        ws = ops.DecodeWorkspace(Bd, Hq, D, math.ceil(8192 / 512), "cuda")
        t = timeit(lambda: ops.paged_decode(qd, kc, vc, bt, ctx, 512, ws))
        byts = 2.0 * Bd * C * Hkv * D * 2
        emit(op="paged-decode", B=Bd, ctx=C, us=round(t * 1e6, 1), gbps=round(byts / t / 1e9))
        del kc, vc


def decode_sweep():
    """Paged decode attention at the bench's decode shape (128 sequences, ~1.2k context, Llama-3-8B
    heads) across partition sizes, with shuffled block tables like the block manager produces."""
    Hq, Hkv, D, bs = 32, 8, 128, 64
    g = torch.Generator().manual_seed(0)
    for Bd in (32, 128, 256):
        ctx_h = torch.randint(1100, 1400, (Bd,), generator=g)
        nbs = [math.ceil(int(c) / bs) for c in ctx_h]
        nbd = sum(nbs)
        kc = torch.randn(nbd, Hkv, bs, D, device="cuda").to(torch.bfloat16)
        vc = torch.randn_like(kc)
        perm = torch.randperm(nbd, generator=g)
        maxb = max(nbs)
        bt = torch.zeros((Bd, maxb), dtype=torch.int32)
        o = 0
        for i, n in enumerate(nbs):
            bt[i, :n] = perm[o:o + n].to(torch.int32)
            o += n
        bt = bt.cuda()
        qd = torch.randn(Bd, Hq, D, device="cuda").to(torch.bfloat16)
        ctx = ctx_h.to(torch.int32).cuda()
        byts = 2.0 * float(ctx_h.sum()) * Hkv * D * 2
        res = {"op": "paged-decode-sweep", "B": Bd, "mean_ctx": int(ctx_h.float().mean())}
        for part in (256, 512, 1024, 2048):
            ws = ops.DecodeWorkspace(Bd, Hq, D, math.ceil(4096 / part), "cuda")
            t = timeit(lambda: ops.paged_decode(qd, kc, vc, bt, ctx, part, ws), iters=50)
            res[f"p{part}_us"] = round(t * 1e6, 1)
            res[f"p{part}_tbps"] = round(byts / t / 1e12, 2)
        emit(**res)
        del kc, vc


def attn_scan():
    """Prefill attention at a fixed 16,384 tokens per launch, T = 256 .. 4096 per sequence, causal and
    full: separates the per-workgroup fixed cost (Q load, first K / V tile, epilogue) from the
    per-tile cost (time = WGs x (F + tiles x c) / slots)."""
    Hq, Hkv, D, bs = 32, 8, 128, 64
    for T in (256, 512, 1024, 2048, 4096):
        B = 16384 // T
        nb = B * T // bs
        kc = torch.randn(nb, Hkv, bs, D, device="cuda").to(torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = torch.arange(nb, dtype=torch.int32, device="cuda").view(B, T // bs)
        q = torch.randn(B * T, Hq, D, device="cuda").to(torch.bfloat16)
        cu = torch.arange(0, B * T + 1, T, dtype=torch.int32, device="cuda")
        ctx = torch.full((B,), T, dtype=torch.int32, device="cuda")
        for causal, pair in ((True, False), (True, True), (True, "q64"), (False, False), (False, "q64")):
            os.environ["DAB_FLASH_PAIR"] = "1" if pair else "0"
            os.environ["DAB_FLASH_Q64"] = "1" if pair == "q64" else "0"
            ts = sorted(timeit(lambda: ops.flash_attention_paged(q, kc, vc, bt, cu, ctx, T, causal=causal))
                        for _ in range(5))
            os.environ.pop("DAB_FLASH_PAIR")
            os.environ.pop("DAB_FLASH_Q64")
            t = ts[2]
            flop = 4.0 * B * Hq * T * T * D / (2 if causal else 1)
            qb = T // 128
            tiles = B * Hq * (sum(2 * (i + 1) for i in range(qb)) if causal else qb * (T // 64))
            emit(op="flash-scan", T=T, B=B, causal=causal, pair=pair, us=round(t * 1e6, 1),
                 tflops=round(flop / t / 1e12, 1),
                 workgroups=B * Hq * qb, wg_tiles=tiles)


def select_suite():
    logits = torch.randn(64, 128256, device="cuda").to(torch.bfloat16)
    temp = torch.ones(64, device="cuda")
    topk = torch.full((64,), 50, dtype=torch.int32, device="cuda")
    topp = torch.full((64,), 0.95, device="cuda")
    cnt = torch.zeros(64, dtype=torch.int64, device="cuda")
    t = timeit(lambda: ops.sample_tokens(logits, temp, topk, topp, 1, cnt))
    emit(op="sample-topk50-topp95-1stage", rows=64, vocab=128256, us=round(t * 1e6, 1))
    ws = ops.kernels.sample_workspace(64, 128256, "cuda")
    t = timeit(lambda: ops.sample_tokens(logits, temp, topk, topp, 1, cnt, fast=True, workspace=ws))
    emit(op="sample-topk50-topp95-2stage", rows=64, vocab=128256, us=round(t * 1e6, 1))
    for R in (128,):
        lg = torch.randn(R, 128256, device="cuda").to(torch.bfloat16) * 2
        t_, k_, p_, c_ = (torch.ones(R, device="cuda"), torch.full((R,), 50, dtype=torch.int32, device="cuda"),
                          torch.full((R,), 0.95, device="cuda"), torch.zeros(R, dtype=torch.int64, device="cuda"))
        ws = ops.kernels.sample_workspace(R, 128256, "cuda")
        t = timeit(lambda: ops.sample_tokens(lg, t_, k_, p_, 1, c_, fast=True, workspace=ws))
        emit(op="sample-topk50-topp95-2stage", rows=R, vocab=128256, us=round(t * 1e6, 1))
    s = torch.randn(64, 1_000_000, device="cuda")
    t = timeit(lambda: ops.topk_rows(s, 250), iters=5)
    emit(op="topk-250", rows=64, n=1_000_000, us=round(t * 1e6, 1), gbps=round(4 * 64e6 / t / 1e9))
    s = torch.randn(64, 1_000_000, device="cuda") * 0.05 + 0.3  # cosine-like: keys share a top byte
    t = timeit(lambda: ops.topk_rows(s, 250), iters=5)
    emit(op="topk-250-cosine-like", rows=64, n=1_000_000, us=round(t * 1e6, 1), gbps=round(4 * 64e6 / t / 1e9))
    x = torch.randn(64, 4096, device="cuda").to(torch.bfloat16)
    w = torch.randn(4096, device="cuda").to(torch.bfloat16)
    t = timeit(lambda: ops.rmsnorm(x, w, 1e-5, residual=x))
    emit(op="rmsnorm+res", rows=64, cols=4096, us=round(t * 1e6, 1))


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which == "stream":
        stream_sweep(sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "all" else None,
                     tuple(int(m) for m in sys.argv[3].split(",")) if len(sys.argv) > 3 else (128,))
    if which == "decode":
        decode_sweep()
    if which in ("all", "gemm"):
        gemm_suite(sys.argv[2] if len(sys.argv) > 2 else None)
    if which in ("all", "attn"):
        attn_suite()
    if which == "attnscan":
        attn_scan()
    if which in ("all", "select"):
        select_suite()
