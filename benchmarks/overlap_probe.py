"""Probe: can compute-bound prefill GEMMs run beside memory-bound decode work on a second stream?

Decode proxy (stream A, normal priority): one Llama-3-8B layer's decode traffic at batch 128 --
gate_up / down / qkv / o projections on hipBLASLt (M = 128, weight-streaming) plus paged decode
attention over 128 x 1.2k contexts -- repeated.  Prefill proxy (stream B, low priority): M = 32K
gate_up GEMMs (compute-bound).  Reports each alone and both together: if the decode proxy slows by
less than the fraction of solo GEMM throughput the prefill keeps, overlapping the next batch's
prefill with the current batch's decode is a net win (an engine design question, not used by the
bench).
"""
import json
import math
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from django_assistant_bot_amd import ops  # noqa: E402


def main():
    dev = "cuda"
    bf = torch.bfloat16
    H, FF, B = 4096, 14336, 128
    ws = [torch.randn(n, k, device=dev, dtype=bf) * 0.02 for n, k in ((6144, H), (H, H), (2 * FF, H), (H, FF))]
    # several layers' worth so the decode proxy streams from HBM, not the 256 MB MALL
    layers = [[w.clone() for w in ws] for _ in range(4)]
    x = torch.randn(B, H, device=dev, dtype=bf)
    xf = torch.randn(B, FF, device=dev, dtype=bf)
    Hq, Hkv, D, bs, C = 32, 8, 128, 64, 1200
    nb = B * math.ceil(C / bs)
    kc = torch.randn(nb, Hkv, bs, D, device=dev, dtype=bf)
    vc = torch.randn_like(kc)
    bt = torch.arange(nb, dtype=torch.int32, device=dev).view(B, -1)
    q = torch.randn(B, Hq, D, device=dev, dtype=bf)
    ctx = torch.full((B,), C, dtype=torch.int32, device=dev)
    wsd = ops.DecodeWorkspace(B, Hq, D, 2, dev)
    Xp = torch.randn(32768, H, device=dev, dtype=bf)
    Wp = torch.randn(2 * FF, H, device=dev, dtype=bf) * 0.02

    def decode_iter():
        for L in layers:
            F.linear(x, L[0])
            ops.paged_decode(q, kc, vc, bt, ctx, 2048, wsd)
            F.linear(x, L[1])
            F.linear(x, L[2])
            F.linear(xf, L[3])

    def prefill_iter():
        F.linear(Xp, Wp)

    # torch: lower number = higher priority; decode gets the high one
    sa = torch.cuda.Stream(priority=-1)
    sb = torch.cuda.Stream(priority=0)
    lo, hi = sb.priority, sa.priority

    def timed(fn, stream, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            e0.record()
            for _ in range(n):
                fn()
            e1.record()
        return e0, e1

    for _ in range(3):
        decode_iter()
        prefill_iter()
    torch.cuda.synchronize()
    nd, npf = 40, 8
    e0, e1 = timed(decode_iter, sa, nd)
    torch.cuda.synchronize()
    dec_solo = e0.elapsed_time(e1) / nd
    e0, e1 = timed(prefill_iter, sb, npf)
    torch.cuda.synchronize()
    pf_solo = e0.elapsed_time(e1) / npf
    # together: prefill GEMMs on the low-priority stream, decode on the other
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # no host sync between the two: both streams hold queued work at once
    p0, p1 = timed(prefill_iter, sb, npf)
    d0, d1 = timed(decode_iter, sa, nd)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    dec_tog = d0.elapsed_time(d1) / nd
    pf_tog = p0.elapsed_time(p1) / npf
    flop = 2.0 * 32768 * H * 2 * FF
    print(json.dumps({"op": "overlap-probe", "decode_iter_ms_solo": round(dec_solo, 3),
                      "decode_iter_ms_together": round(dec_tog, 3), "prefill_gemm_ms_solo": round(pf_solo, 3),
                      "prefill_gemm_ms_together": round(pf_tog, 3),
                      "prefill_tflops_solo": round(flop / pf_solo / 1e9, 1),
                      "wall_ms_together": round(wall, 1),
                      "serial_ms": round(nd * dec_solo + npf * pf_solo, 1),
                      "stream_priorities": [lo, hi]}), flush=True)
    # CU-masked streams: prefill on a quarter of the CUs, decode on the rest
    nat = ops.native()
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (n_cu + 31) // 32
    for pattern in ("interleaved", "contiguous"):
        for frac in (4, 8):
            pf_cus = [i for i in range(n_cu) if (i % frac == 0 if pattern == "interleaved" else i < n_cu // frac)]
            mp, md = [0] * words, [0] * words
            for i in range(n_cu):
                if i in pf_cus:
                    mp[i // 32] |= 1 << (i % 32)
                else:
                    md[i // 32] |= 1 << (i % 32)
            hp, hd = nat.create_cu_masked_stream(mp), nat.create_cu_masked_stream(md)
            sp, sd = torch.cuda.ExternalStream(hp), torch.cuda.ExternalStream(hd)
            torch.cuda.synchronize()
            e0, e1 = timed(decode_iter, sd, nd)
            torch.cuda.synchronize()
            dec_mask_solo = e0.elapsed_time(e1) / nd
            t0 = time.perf_counter()
            p0, p1 = timed(prefill_iter, sp, npf)
            d0, d1 = timed(decode_iter, sd, nd)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3
            print(json.dumps({"op": "overlap-cumask", "pattern": pattern, "prefill_cus": len(pf_cus),
                              "decode_iter_ms_solo_all_cus": round(dec_solo, 3),
                              "decode_iter_ms_solo_masked": round(dec_mask_solo, 3),
                              "decode_iter_ms_together": round(d0.elapsed_time(d1) / nd, 3),
                              "prefill_gemm_ms_together": round(p0.elapsed_time(p1) / npf, 3),
                              "prefill_gemm_ms_solo_all_cus": round(pf_solo, 3),
                              "wall_ms_together": round(wall, 1)}), flush=True)
            nat.destroy_stream(hp)
            nat.destroy_stream(hd)


if __name__ == "__main__":
    main()
