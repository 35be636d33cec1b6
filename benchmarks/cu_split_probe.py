"""Probe: prefill on one CU partition beside the running decode on the rest (real engine kernels).

Decode: the production Llama-3-8B engine at batch 128 (~1.1k-token contexts, HIP-graph decode with
the streaming GEMMs and the paged attention), stepped on a CU-masked stream D.  Prefill: the same
model's forward over a packed chunk of 8 x 1024-token prompts (gemm256 projections, flash
attention into a scratch KV cache, last-token logits) on a CU-masked stream P.  For each split the
probe times each side alone on its partition and both together, and projects the serving rate if
every question's prompt is prefilled on P while D keeps decoding: a question costs
max(255 decode steps / 128 rows, 1092 prompt tokens / P's token rate).

    python benchmarks/cu_split_probe.py [--splits 64,96,128] [--patterns contig,xcd]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def masks(n_cu: int, n_p: int, pattern: str):
    """(P words, D words) of a split: ``contig`` = CUs 0..n_p-1 to P; ``xcd`` = the first n_p / 8 CUs
    of every 32-CU block (one block per XCD if the mask numbers CUs XCD by XCD); ``mod8`` = CU i to P
    when (i // 8) % (n_cu // n_p) == 0 (if the mask interleaves XCDs CU by CU)."""
    words = (n_cu + 31) // 32
    mp_, md = [0] * words, [0] * words
    per = n_cu // 8
    for i in range(n_cu):
        if pattern == "contig":
            to_p = i < n_p
        elif pattern == "xcd":
            to_p = (i % per) < n_p // 8
        else:
            to_p = (i // 8) % (n_cu // n_p) == 0
        (mp_ if to_p else md)[i // 32] |= 1 << (i % 32)
    return mp_, md


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splits", default="64,96,128")
    ap.add_argument("--patterns", default="contig,xcd")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--prompt", type=int, default=1100)
    ap.add_argument("--chunk-seqs", type=int, default=8)
    ap.add_argument("--chunk-len", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--chunks", type=int, default=3)
    args = ap.parse_args()
    from django_assistant_bot_amd import ops
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine, SamplingParams
    from django_assistant_bot_amd.models.llama import AttnMeta, KVCache

    torch.manual_seed(0)
    eng = LLMEngine("llama-3-8b", device="cuda", max_batch=args.batch, kv_cache_gb=60, max_prefill_tokens=32768)
    g = torch.Generator().manual_seed(1)
    sp = SamplingParams(max_new_tokens=100000, ignore_eos=True)
    for _ in range(args.batch):
        eng.add_request(torch.randint(0, 128000, (args.prompt,), generator=g).tolist(), sp)
    while eng.waiting or eng.prefilling or eng._pending_prefill is not None:
        eng.step()
    for _ in range(4):
        eng.step()
    eng._finish_inflight()
    # prefill chunk on a scratch cache
    cfg, m = eng.cfg, eng.model
    S, L = args.chunk_seqs, args.chunk_len
    T = S * L
    nb = S * (L // 64)
    kv2 = KVCache(cfg.layers, nb, cfg.kv_heads, 64, cfg.head_dim, "cuda")
    i32 = dict(dtype=torch.int32, device="cuda")
    ids = torch.randint(0, 128000, (T,), **i32)
    meta = AttnMeta(decode=False, positions=torch.arange(L, **i32).repeat(S), slots=torch.arange(T, device="cuda"),
                    block_tables=torch.arange(nb, **i32).view(S, L // 64), ctx_lens=torch.full((S,), L, **i32),
                    cu_q=torch.arange(0, T + 1, L, **i32), max_q=L)
    last = torch.arange(L - 1, T, L, device="cuda")

    def prefill():
        h = m.forward(ids, meta, kv2)
        m.logits(h.index_select(0, last))

    def decode_steps(n):
        t0 = time.perf_counter()
        for _ in range(n):
            eng.step()
        eng._finish_inflight()
        torch.cuda.current_stream().synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    def prefill_chunks(k, stream):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            e0.record()
            for _ in range(k):
                prefill()
            e1.record()
        return e0, e1

    prefill()
    torch.cuda.synchronize()
    out = {"op": "cu-split-probe"}
    out["decode_ms_full"] = round(decode_steps(args.steps), 3)
    e0, e1 = prefill_chunks(args.chunks, torch.cuda.current_stream())
    torch.cuda.synchronize()
    out["prefill_ms_full"] = round(e0.elapsed_time(e1) / args.chunks, 2)
    out["prefill_tokens"] = T
    print(json.dumps(out), flush=True)
    nat = ops.native()
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    base_q = 1.0 / (255 * out["decode_ms_full"] / 128 + 1092 * out["prefill_ms_full"] / T) * 1e3
    print(json.dumps({"op": "serial-baseline", "q_per_s": round(base_q, 2)}), flush=True)
    for pattern in args.patterns.split(","):
        for n_p in [int(x) for x in args.splits.split(",")]:
            mp_, md = masks(n_cu, n_p, pattern)
            hp, hd = nat.create_cu_masked_stream(mp_), nat.create_cu_masked_stream(md)
            sp_, sd = torch.cuda.ExternalStream(hp), torch.cuda.ExternalStream(hd)
            eng._graphs.clear()  # graphs re-captured with the new stream in effect
            with torch.cuda.stream(sd):
                decode_steps(4)
                d_solo = decode_steps(args.steps)
            e0, e1 = prefill_chunks(args.chunks, sp_)
            torch.cuda.synchronize()
            p_solo = e0.elapsed_time(e1) / args.chunks
            # together: the prefill chunks are queued on P first, then D steps while they run
            e0, e1 = prefill_chunks(args.chunks, sp_)
            with torch.cuda.stream(sd):
                n_d = 0
                t0 = time.perf_counter()
                while not e1.query() or n_d < 4:
                    eng.step()
                    n_d += 1
                eng._finish_inflight()
                sd.synchronize()
                d_tog = (time.perf_counter() - t0) / n_d * 1e3
            torch.cuda.synchronize()
            p_tog = e0.elapsed_time(e1) / args.chunks
            d_q = 255 * d_tog / 128
            p_q = 1092 * p_tog / T
            res = {"op": "cu-split", "pattern": pattern, "prefill_cus": n_p, "decode_ms_solo_masked": round(d_solo, 3),
                   "prefill_ms_solo_masked": round(p_solo, 2), "decode_ms_together": round(d_tog, 3),
                   "prefill_ms_together": round(p_tog, 2), "decode_steps_together": n_d,
                   "ms_per_query_decode": round(d_q, 2), "ms_per_query_prefill": round(p_q, 2),
                   "projected_q_per_s": round(1e3 / max(d_q, p_q), 2)}
            print(json.dumps(res), flush=True)
            torch.cuda.synchronize()
            nat.destroy_stream(hp)
            nat.destroy_stream(hd)


if __name__ == "__main__":
    main()
