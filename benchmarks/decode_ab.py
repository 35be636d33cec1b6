"""Interleaved A/B of decode-step variants inside ONE engine (un-profiled wall time per step).

rocprof serialises kernels and shifts the clock, so small decode changes can rank differently
under it than in the bench (profiles/round3_layout_and_parity.md: a fused prologue that won under
rocprof lost 0.18 ms per step without it).  This harness builds the bench's decode state once
(Llama-3-8B, 128 sequences of ~1.1k-token prompts, pipelined HIP-graph decode), then times each
arm for ``--steps`` decode steps, arms interleaved over ``--rounds`` rounds, with graphs
re-captured per arm and every arm starting from the same contexts (prefix-cache re-admission).  An arm sets per-projection
(stream_gemm cfg, K-slices) overrides (``TunedLlama``: a subclass of the production model whose
``_stream_choice`` consults them) and/or the decode attention partition.

    python benchmarks/decode_ab.py --arms base,qkv21,o4 --rounds 3 --steps 40
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ARMS = {
    "base": {},
    "qkv21": {"qkv": (21, 4)},
    "qkv23": {"qkv": (23, 4)},
    "qkv14": {"qkv": (14, 4)},
    "qkv2": {"qkv": (10, 2)},
    "o4": {"o": (10, 4)},
    "o16": {"o": (10, 16)},
    "o14": {"o": (14, 8)},
    "down4": {"down": (10, 4)},
    "down14": {"down": (14, 8)},
    "down15": {"down": (15, 8)},
    "gu22": {"gate_up": (22, 1)},
    "gu10": {"gate_up": (10, 1)},
    "lm29": {"lm_head": (29, 1)},
    "lm10": {"lm_head": (10, 1)},
    "gu14": {"gate_up": (14, 1)},
    "gu15": {"gate_up": (15, 1)},
    "qkv15": {"qkv": (15, 4)},
    "o15": {"o": (15, 8)},
    "o9_4": {"o": (9, 4)},
    "o11_4": {"o": (11, 4)},
    "down9_4": {"down": (9, 4)},
    "down11_4": {"down": (11, 4)},
    "qkv9_2": {"qkv": (9, 2)},
    "od9_4": {"o": (9, 4), "down": (9, 4)},
    # batch 65-128: narrow tiles at 2 K-slices (stream_gemm cfg 34 BN 32, 35 BN 48)
    "o34_2": {"o": (34, 2)},
    "down34_2": {"down": (34, 2)},
    "qkv35_2": {"qkv": (35, 2)},
    "narrow": {"o": (34, 2), "down": (34, 2), "qkv": (35, 2)},
    # batch 65-128: two workgroups per CU (cfg 36 / 37, BN 64, 2-stage X ring)
    "o36_8": {"o": (36, 8)},
    "down36_8": {"down": (36, 8)},
    "qkv36_4": {"qkv": (36, 4)},
    "qkv36_8": {"qkv": (36, 8)},
    "o37_8": {"o": (37, 8)},
    "down37_8": {"down": (37, 8)},
    "occ2": {"o": (36, 8), "down": (36, 8), "qkv": (36, 4)},
    "part1024": {"_part": 1024},
    "part512": {"_part": 512},
    "m16via13": {"_m16": 13},                # batches <= 16 on the M <= 64 configuration (cfg 13)
    "m32via13": {"_m32": 13},                # batches 17..32 on cfg 13
    "spart256": {"_spart": 256},            # small-batch partition (engine.part_size; ctx <= 16 x part)
    "spart128": {"_spart": 128},
    "part640": {"_part": 640},              # ~2 equal partitions of a ~1.2k context
    "part768": {"_part": 768},
    # batches <= 16: the consumer-side RMSNorm (``_layer_small``) instead of the norm launches
    "normfused": {"_fuse": True},
    # ... with the o / down residual producers at 32 weight rows per workgroup (cfg 33)
    "res32": {"_fuse": True, "_res_cfg": 33},
    # batches <= 16: Infinity-Cache warm-up of the next o / gate_up weights riding on the attention
    "warm32": {"_warm": 32},
    "warm64": {"_warm": 64},
    "warm96": {"_warm": 96},
    "warm160": {"_warm": 160},
    "warm96b128": {"_warm": 96, "_warm_blocks": 128},
    # split-K launches with S % 8 == 0 (o / down at batch 128): K-slices grouped per XCD instead of
    # tiles, so an XCD's L2 holds 1/8 of X
    "slicexcd": {"_slice_xcd": 1},
    # bf16 split-K slabs (LlamaModel.slab_bf16) against fp32
    "slab16": {"_slab16": True},
    # split counts re-tuned for bf16 slabs
    "qkv8": {"qkv": (10, 8)},
    "down16": {"down": (10, 16)},
    "o4b": {"o": (10, 4)},
    "slab32": {"_slab16": False},
    # projection copies in the plain / grouped fragment layout (shuffle_weights(w, G), LlamaModel.PROJ_GROUPS)
    "gu_g1": {"_groups": {"gate_up": 1}},
    "all_g8": {"_groups": {"qkv": 8, "o": 8, "down": 8}},
    "down_g8": {"_groups": {"down": 8}},
    "qkvo_g8": {"_groups": {"qkv": 8, "o": 8}},
    "gu27": {"gate_up": (27, 1)},  # batches 129..256: gate_up on the M <= 256 streaming tiles (round-6 default: gemm_mid)
    "gu41": {"gate_up": (41, 1)},
    "gu42": {"gate_up": (42, 1)},
}


def tuned_model_class():
    from django_assistant_bot_amd.models.llama import LlamaModel

    class TunedLlama(LlamaModel):
        """The production decoder with per-projection (stream_gemm cfg, K-slices) overrides."""

        overrides: dict = {}

        def _stream_choice(self, name, M, N, K):
            if name in self.overrides:
                return self.overrides[name]
            return super()._stream_choice(name, M, N, K)

    return TunedLlama


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", default="base,qkv21,o4,down14")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--prompt", type=int, default=1100)
    ap.add_argument("--block-size", type=int, default=64, help="paged-KV block (tokens): one engine per value")
    args = ap.parse_args()
    from django_assistant_bot_amd import ops
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine, SamplingParams

    torch.manual_seed(0)
    eng = LLMEngine("llama-3-8b", device="cuda", max_batch=args.batch, kv_cache_gb=120, max_prefill_tokens=32768,
                    block_size=args.block_size)
    eng.model.__class__ = tuned_model_class()  # same object, overridable stream choice
    g = torch.Generator().manual_seed(1)
    sp = SamplingParams(max_new_tokens=6000, ignore_eos=True)
    prompts = [torch.randint(0, 128000, (args.prompt + int(torch.randint(-100, 100, (1,), generator=g)),),
                             generator=g).tolist() for _ in range(args.batch)]

    def restart():
        """Every arm decodes from the same contexts: drop the batch and re-admit the same prompts
        (their blocks come back from the prefix cache, so only the last partial block re-runs)."""
        eng._finish_inflight()
        for r in [r.rid for r in list(eng.running) + list(eng.prefilling) + list(eng.waiting)]:
            eng.abort(r)
        eng.finished.clear()
        for p in prompts:
            eng.add_request(p, sp)
        while eng.waiting or eng.prefilling or eng._pending_prefill is not None:
            eng.step()

    base_part, base_spart = eng.long_part_size, eng.part_size
    base_groups = dict(eng.model.proj_group)
    arms = args.arms.split(",")
    res = {a: [] for a in arms}
    for r in range(args.rounds):
        for a in arms:
            spec = dict(ARMS[a])
            restart()
            eng.model.overrides = {k: v for k, v in spec.items() if not k.startswith("_")}
            eng.long_part_size = spec.get("_part", base_part)
            eng.part_size = spec.get("_spart", base_spart)
            eng.model.STREAM_CFG_M16 = spec.get("_m16", type(eng.model).STREAM_CFG_M16)
            eng.model.STREAM_CFG_M32 = spec.get("_m32", type(eng.model).STREAM_CFG_M32)
            eng.model.small_norm_fused = spec.get("_fuse", False)
            if eng.model.small_norm_fused:
                # random init: unit RMSNorm gains, so the weights are already "folded" (W diag(1) = W)
                assert all(bool(torch.all(L.attn_norm == 1)) and bool(torch.all(L.mlp_norm == 1))
                           for L in eng.model.layers)
                eng.model.fold_norms = eng.model.frag
            eng.model.l3_warm_mb = spec.get("_warm", type(eng.model).l3_warm_mb)
            eng.model.l3_warm_blocks = spec.get("_warm_blocks", type(eng.model).l3_warm_blocks)
            eng.model.STREAM_CFG_RES16 = spec.get("_res_cfg", type(eng.model).STREAM_CFG_RES16)
            ops.native().stream_gemm_set_slice_xcd(spec.get("_slice_xcd", 0))
            eng.model.slab_bf16 = spec.get("_slab16", type(eng.model).slab_bf16)
            for n, g in {**base_groups, **spec.get("_groups", {})}.items():
                eng.model.set_proj_group(n, g)
            eng._graphs.clear()
            for _ in range(4):
                eng.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                eng.step()
            eng._finish_inflight()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / args.steps * 1e3
            res[a].append(round(ms, 4))
            print(json.dumps({"round": r, "arm": a, "ms_per_step": round(ms, 4)}), flush=True)
    base = sorted(res[arms[0]])[len(res[arms[0]]) // 2]
    for a in arms:
        med = sorted(res[a])[len(res[a]) // 2]
        print(json.dumps({"arm": a, "median_ms": med, "vs_first": round(med / base, 4), "all": res[a]}), flush=True)


if __name__ == "__main__":
    main()
