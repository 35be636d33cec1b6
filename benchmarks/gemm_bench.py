"""Large-M GEMM study: native gemm256 (8-phase 256x256, gemm256.hip) vs hipBLASLt (F.linear) on the
prefill / encoder shapes, bf16, uniform random [-1, 1) operands (cdna_hip_programming.md rule 25).

For each shape: numerics of the native kernel against an fp32 PyTorch reference on a row sample,
then interleaved timing rounds in one process (rule 24): native, library, native, library, ...
The library arm includes the separate elementwise pass the native epilogue fuses (SwiGLU: hipBLASLt
+ silu_mul; GELU: hipBLASLt + bias/GELU pass), so ``speedup`` compares what a layer actually runs.

    python benchmarks/gemm_bench.py [--shapes llama,bge,square] [--rounds 5] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from django_assistant_bot_amd import ops  # noqa: E402

SHAPES = {
    "llama": [("llama8b-qkv", 32768, 6144, 4096, "none"), ("llama8b-o", 32768, 4096, 4096, "none"),
              ("llama8b-gateup", 32768, 28672, 4096, "swiglu"), ("llama8b-down", 32768, 4096, 14336, "none")],
    "bge": [("bge-qkv", 65536, 2304, 768, "bias"), ("bge-o", 65536, 768, 768, "bias"),
            ("bge-up", 65536, 3072, 768, "gelu"), ("bge-down", 65536, 768, 3072, "bias")],
    "square": [("sq4096", 4096, 4096, 4096, "none"), ("sq8192", 8192, 8192, 8192, "none")],
    "edge": [("edge-m1000", 1000, 1024, 512, "none"), ("edge-m300", 300, 512, 256, "bias")],
    # mixed prefill + decode steps: M = 384 / 640 / 1024 tokens per step
    "mid": [(f"mid{M}-{n}", M, N, K, kind) for M in (384, 512, 640, 768, 1024, 2048)
            for n, N, K, kind in (("qkv", 6144, 4096, "none"), ("o", 4096, 4096, "none"),
                                  ("gateup", 28672, 4096, "swiglu"), ("down", 4096, 14336, "none"))],
}


def roofline_us(M, N, K):
    """max(weight bytes / 6 TB/s, FLOPs / 1.5 PF/s): the mid-M target of VERDICT r4 item 1."""
    return max(2.0 * N * K / 6e12, 2.0 * M * N * K / 1.5e15) * 1e6


def rand(shape, scale=1.0):
    return ((torch.rand(shape, device="cuda") * 2 - 1) * scale).to(torch.bfloat16)


EPI = {"none": ops.EPI_NONE, "bias": ops.EPI_NONE, "gelu": ops.EPI_GELU, "swiglu": ops.EPI_SWIGLU8}


def run_native(a, w, b, kind, out, shuffled):
    """The layer's own call: the decoder keeps every projection in the fragment layout
    (``shuffle_weights``) and gate/up interleaved in 8-row groups (EPI_SWIGLU8)."""
    return ops.gemm_bt(a, w, bias=b if kind in ("bias", "gelu") else None, epilogue=EPI[kind], out=out,
                       shuffled=shuffled)


def run_lib(a, w, b, kind):
    if kind == "none":
        return F.linear(a, w)
    if kind == "bias":
        return F.linear(a, w, b)
    if kind == "gelu":
        return ops.gelu(F.linear(a, w), b)
    return ops.silu_mul(F.linear(a, w), interleaved=True)


def check(a, w, b, kind, out, rows):
    idx = torch.cat([torch.arange(0, min(rows, a.shape[0]), device="cuda"),
                     torch.arange(max(0, a.shape[0] - rows), a.shape[0], device="cuda")]).unique()
    ref = ops.reference.gemm_bt(a[idx], w, b if kind in ("bias", "gelu") else None, None, EPI[kind],
                                out_f32=True)
    got = out[idx].float()
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    return err, scale


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="llama,bge,square,edge")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--native-only", action="store_true", help="profile mode: only the native arm")
    ap.add_argument("--only", default="", help="comma list of op names to run")
    ap.add_argument("--mid-variants", action="store_true", help="gemm_mid A/B arms (BK 64, no combine)")
    ap.add_argument("--ab-layout", action="store_true",
                    help="llama shapes: also time the row-major weight layout (arm 'rowmajor')")
    args = ap.parse_args()
    torch.manual_seed(0)
    for group in args.shapes.split(","):
        for name, M, N, K, kind in SHAPES[group]:
            if args.only and name not in args.only.split(","):
                continue
            a = rand((M, K))
            w = rand((N, K), 0.05)
            b = rand((N,), 0.5)
            n_out = N // 2 if kind == "swiglu" else N
            out = torch.empty((M, n_out), dtype=torch.bfloat16, device="cuda")
            frag = group in ("llama", "mid")
            ws = ops.shuffle_weights(w) if frag else w
            run_native(a, ws, b, kind, out, frag)
            torch.cuda.synchronize()
            err, scale = check(a, w, b, kind, out, 256)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            extra = {}
            nat, lib = [], []
            arms = [("nat", lambda: run_native(a, ws, b, kind, out, frag)), ("lib", lambda: run_lib(a, w, b, kind))]
            if args.native_only:
                arms = arms[:1]
            if group == "mid" and frag and ops.native().gemm256_ok(M, N, K, K, K):
                arms.append(("g256", lambda: ops.kernels.gemm256(a, ws, epilogue=EPI[kind], shuffled=True)))
            if frag and kind in ("none", "swiglu") and ops.kernels.gemm_mid_ok(M, N, K, K):
                # the mid-M stream-K kernel (gemm_mid.hip), checked against the same reference first
                gm_out = ops.kernels.gemm_mid(a, ws, epilogue=EPI[kind])
                torch.cuda.synchronize()
                extra["gmid_err"] = [check(a, w, b, kind, gm_out, 256)[0]]
                arms.append(("gmid", lambda: ops.kernels.gemm_mid(a, ws, epilogue=EPI[kind], out=out)))
                if args.mid_variants:
                    for v in (64, 1032, 1064):  # BK 64; split tiles left uncombined (timing only)
                        arms.append((f"gmid{v}", lambda v=v: ops.kernels.gemm_mid(a, ws, epilogue=EPI[kind], out=out,
                                                                                  variant=v)))
            if args.ab_layout and frag:
                arms.append(("rowmajor", lambda: run_native(a, w, b, kind, out, False)))
            for _ in range(args.rounds):
                for arm, fn in arms:
                    fn()
                    ev[0].record()
                    for _ in range(args.iters):
                        fn()
                    ev[1].record()
                    torch.cuda.synchronize()
                    t = ev[0].elapsed_time(ev[1]) / args.iters * 1e3
                    extra.setdefault(arm, []).append(t) if arm not in ("nat", "lib") else \
                        {"nat": nat, "lib": lib}[arm].append(t)
            nat.sort()
            lib.sort()
            lib = lib or [float("nan")]
            flop = 2.0 * M * N * K
            tn, tl = nat[len(nat) // 2], lib[len(lib) // 2]
            print(json.dumps({"op": name, "M": M, "N": N, "K": K, "epilogue": kind,
                              "native_us": round(tn, 1), "native_min_us": round(nat[0], 1),
                              "lib_us": round(tl, 1), "lib_min_us": round(lib[0], 1),
                              "native_tflops": round(flop / tn / 1e6, 1), "lib_tflops": round(flop / tl / 1e6, 1),
                              "speedup": round(tl / tn, 3), "max_abs_err": round(err, 5),
                              "ref_max": round(scale, 3), "ok": err <= 0.02 * max(scale, 1.0),
                              "roofline_us": round(roofline_us(M, N, K), 1),
                              "vs_roofline": round(tn / roofline_us(M, N, K), 3),
                              **{(k if k.endswith("_err") else f"{k}_us"): round(sorted(v)[len(v) // 2], 4 if k.endswith("_err") else 1)
                                 for k, v in extra.items()}}),
                  flush=True)
            del a, w, ws, b, out
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
