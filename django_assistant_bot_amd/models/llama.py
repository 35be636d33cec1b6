"""Llama-3 family decoder on the native kernels with a paged KV cache and tensor parallelism.

Replaces HF ``AutoModelForCausalLM.generate`` of the reference (ai/providers/transformers.py:35-94).
One forward serves both phases:

  * prefill (packed variable-length prompt chunks; flash attention reads K/V from the paged cache,
    so chunked prefill and cached shared prefixes need no special path);
  * decode (one token per running sequence; split-K paged decode attention), capturable in a HIP
    graph because every op enqueues on the current stream with fixed shapes.

Per layer:  RMSNorm(+residual) -> QKV GEMM -> RoPE + KV-cache write -> attention -> O GEMM
[-> TP all-reduce] -> RMSNorm(+residual) -> gate|up GEMM (+fused SwiGLU) -> down GEMM
[-> TP all-reduce].  Under TP each rank owns Hq/tp query heads, Hkv/tp KV heads and F/tp MLP
columns (Megatron split); the two all-reduces per layer run on the RCCL process group.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch

from .. import ops
from ..ops import reference as ref
from .configs import DecoderConfig


@dataclass
class DecoderLayer:
    attn_norm: torch.Tensor
    qkv_w: torch.Tensor
    o_w: torch.Tensor
    mlp_norm: torch.Tensor
    gate_up_w: torch.Tensor
    down_w: torch.Tensor
    # decode copies in the ops.shuffle_weights layout (warp-specialised streaming kernel), or None
    qkv_ws: torch.Tensor | None = None
    o_ws: torch.Tensor | None = None
    gate_up_ws: torch.Tensor | None = None
    down_ws: torch.Tensor | None = None


@dataclass
class AttnMeta:
    """Per-forward batch description (device tensors, fixed shapes in decode graphs)."""

    decode: bool
    positions: torch.Tensor  # int32 [T]
    slots: torch.Tensor  # int64 [T] cache slot of each token (<0 = padding)
    block_tables: torch.Tensor  # int32 [B, max_blocks]
    ctx_lens: torch.Tensor  # int32 [B] total tokens in cache after this step
    cu_q: torch.Tensor | None = None  # int32 [B+1] (prefill)
    max_q: int = 1
    workspace: ops.DecodeWorkspace | None = None
    part_size: int = 512
    # mixed step: the LAST n_decode tokens are single-token decode rows (one per sequence) with their
    # own block tables / context lengths; the tokens before them are prefill chunks described above
    n_decode: int = 0
    dec_block_tables: torch.Tensor | None = None
    dec_ctx_lens: torch.Tensor | None = None
    order: torch.Tensor | None = None  # int32 [B] decode attention dispatch order (longest context first)


class KVCache:
    """Paged KV cache: per layer [num_blocks, Hkv_local, block_size, D] for K and for V."""

    def __init__(self, layers, num_blocks, kv_heads, block_size, head_dim, device, dtype=torch.bfloat16):
        self.num_blocks, self.block_size = num_blocks, block_size
        self.k = torch.zeros((layers, num_blocks, kv_heads, block_size, head_dim), device=device, dtype=dtype)
        self.v = torch.zeros_like(self.k)

    @staticmethod
    def bytes_per_block(layers, kv_heads, block_size, head_dim, dtype=torch.bfloat16):
        return 2 * layers * kv_heads * block_size * head_dim * torch.finfo(dtype).bits // 8


class LlamaModel:
    def __init__(self, cfg: DecoderConfig, weights: dict, device, tp_group=None, tp_size: int = 1,
                 interleaved_mlp: bool = False):
        self.cfg = cfg
        self.device = torch.device(device)
        self.tp_group, self.tp_size = tp_group, tp_size
        self.hq = cfg.heads // tp_size
        self.hkv = cfg.kv_heads // tp_size
        self.interleaved_mlp = interleaved_mlp
        w = {k: v.to(self.device) for k, v in weights.items()}
        self.embed = w["embed"]
        self.final_norm = w["final_norm"]
        self.lm_head = w.get("lm_head", self.embed)
        self.layers = [
            DecoderLayer(*(w[f"l{i}.{n}"] for n in ("attn_norm", "qkv_w", "o_w", "mlp_norm", "gate_up_w", "down_w")))
            for i in range(cfg.layers)
        ]
        # decode projections on the weight-streaming kernel: "all", "none", or a comma list of
        # qkv,o,gate_up,down,lm_head.  Default o,down: split-K beats hipBLASLt there at M 64-128
        # (o 16.6 vs 24.1 us, down 39.7 vs 48+ us at M=128; decode step 9.50 -> 9.23 ms at batch 128),
        # ties on qkv and loses on gate_up (profiles/decode_gemm_m128_study.md)
        sel = os.environ.get("DAB_SKINNY", "o,down")
        sel = {"1": "all", "0": "none"}.get(sel, sel)
        names = ("qkv", "o", "gate_up", "down", "lm_head")
        self.skinny_for = set(names) if sel == "all" else set() if sel == "none" else set(sel.split(","))
        self.use_skinny = bool(self.skinny_for)
        self._split_cache: dict = {}
        # decode projections on the warp-specialised streaming kernel (stream_gemm.hip) over weight
        # copies in the coalesced shuffle_weights layout: qkv 25.6 -> 16.9 us, o 16.6 -> 14.0, down
        # 39.7 -> 29.2, gate_up 51.8 + 5.1 (SiLU) -> 53.0 with SwiGLU fused, at M = 128
        # (profiles/decode_stream_gemm.md).  DAB_DECODE_GEMM=skinny keeps the split-K kernel above.
        self.stream = False
        self.lm_head_ws = None
        if (os.environ.get("DAB_DECODE_GEMM", "stream") == "stream" and self.device.type == "cuda"
                and self.use_skinny):
            self.stream = self._make_stream_copies()

        self.custom_ar = None  # parallel.custom_allreduce.CustomAllReduce (set by the engine)
        inv = ref.llama3_inv_freq(cfg.head_dim, cfg.rope_theta, cfg.rope_scaling)
        self.cos_sin = ref.rope_cos_sin(inv, cfg.max_position).to(self.device)

    @property
    def dtype(self):
        return self.embed.dtype

    def _all_reduce(self, x):
        """TP partial sums: the one-shot IPC all-reduce for decode-sized messages when the engine
        attached one (``custom_ar``), RCCL otherwise (prefill, CPU/gloo)."""
        if self.tp_size > 1:
            ar = self.custom_ar
            if ar is not None and ar.eligible(x):
                return ar.all_reduce(x)
            import torch.distributed as dist

            dist.all_reduce(x, group=self.tp_group)
        return x

    STREAM_CFG_M64, STREAM_CFG_M128 = 13, 10  # stream_gemm.hip configurations (BN 128, shuffled)
    # whole-chip tiling at M 65..128 (one 16-row tile per compute wave): gate_up's 28672 rows / 112
    # make exactly 256 workgroups where BN 128 left 32 of the 256 CUs idle: 54.9 -> 51.5 us cold
    # (kernel_bench stream).  qkv at 96 rows x 4 K-slices (cfg 21, also 256 workgroups) measured
    # slower than BN 128 x 4 (17.1 vs 15.8 us) and stays on cfg 10.  DAB_STREAM_WIDE=0: BN 128 (A/B).
    # The LM head at M 65..128 uses 192-row tiles (6 compute waves): 2/3 of the X staging per
    # weight byte, 228.7 -> 221.3 us (kernel_bench stream lm_head, cold weights).
    STREAM_WIDE = {"gate_up": 20, "lm_head": 28}
    _wide = os.environ.get("DAB_STREAM_WIDE", "1") != "0"

    @staticmethod
    def _stream_ok(w: torch.Tensor) -> bool:
        return w.shape[0] % 128 == 0 and w.shape[1] % 128 == 0

    # decode batches of 129..256 rows: 64-row tiles, 2 k-groups x 4 row groups (cfg 27; M = 256, cold
    # weights: qkv 27.4 / o 18.6 / gate_up 98.7 / down 49.2 us against 32.4 / 25.8 / 104 / 55 for two
    # M = 128 passes, profiles/decode_round2.md), so the step no longer falls back to the large-M GEMM
    STREAM_CFG_M256 = 27
    STREAM_MAX_M = 256

    def _stream_cfg(self, name: str, M: int, N: int) -> int:
        if M > 128:
            return self.STREAM_CFG_M256
        if M <= 64:
            return self.STREAM_CFG_M64
        cfg = self.STREAM_WIDE.get(name) if self._wide else None
        if cfg is not None and N % ops.native().stream_gemm_bn(cfg) == 0:
            return cfg
        return self.STREAM_CFG_M128

    def _make_stream_copies(self) -> bool:
        """Shuffled decode copies of the projection weights (and of the LM head, which decode and
        the prefill last-token logits stream at M <= 128) when they fit comfortably (each copy is
        the size of the weights; the KV pool is sized from what is left).  The gate_up copy is
        regrouped to 8-row [gate | up] pairs (EPI_SWIGLU8) so any 16-row multiple tiles it."""
        names = ("qkv", "o", "gate_up", "down") if self.interleaved_mlp else ("qkv", "o", "down")
        mats = [(L, n) for L in self.layers for n in names if self._stream_ok(getattr(L, f"{n}_w"))]
        extra = sum(getattr(L, f"{n}_w").numel() * 2 for L, n in mats)
        head = self._stream_ok(self.lm_head)
        extra += self.lm_head.numel() * 2 if head else 0
        free, _ = torch.cuda.mem_get_info(self.device)
        if not mats or extra > 0.4 * free:
            return False
        for L, n in mats:
            w = getattr(L, f"{n}_w")
            if n == "gate_up":
                w = ops.regroup_gate_up(w, 16, 8)
            setattr(L, f"{n}_ws", ops.shuffle_weights(w))
        if head:
            self.lm_head_ws = ops.shuffle_weights(self.lm_head)
        return True

    @staticmethod
    def _stream_splits(N: int, K: int, bn: int = 128) -> int:
        """K-slices for stream_gemm: the fewest that give >= 192 workgroups of ``bn`` weight rows."""
        tiles, best = N // bn, 1
        for s in (1, 2, 4, 8, 16):
            if K % (128 * s):
                break
            best = s
            if tiles * s >= 192:
                break
        return best

    def _splits(self, w: torch.Tensor) -> int:
        key = id(w)
        s = self._split_cache.get(key)
        if s is None:
            s = self._split_cache[key] = ops.skinny_splits(w.shape[0], w.shape[1])
        return s

    def _proj(self, x, w, sk: bool, allow_slabs: bool = True, name: str = "", ws=None):
        """Projection of the decode (``sk``: weight-streaming kernel, fp32 split-K slabs when the
        consumer can sum them) or prefill path (native MFMA GEMM: the 256x256 8-phase kernel for
        large token counts, ``gemm256.hip``)."""
        if sk and ws is not None:
            cfg = self._stream_cfg(name, x.shape[0], w.shape[0])
            s = self._stream_splits(w.shape[0], w.shape[1], ops.native().stream_gemm_bn(cfg))
            out = ops.stream_gemm(x, ws, splits=s, cfg=cfg, nt=True)
            return ops.skinny_reduce(out) if (s > 1 and not allow_slabs) else out
        if not sk or name not in self.skinny_for or x.shape[0] > ops.SKINNY_MAX_M:
            return ops.gemm_bt(x, w) if x.is_cuda else ops.linear(x, w)
        s = self._splits(w)
        if s > 1 and not allow_slabs:
            return ops.skinny_reduce(ops.skinny_gemm(x, w, splits=s))
        return ops.skinny_gemm(x, w, splits=s)

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: KVCache) -> torch.Tensor:
        """ids int32 [T] -> final hidden states [T, H] (after the last RMSNorm)."""
        cfg = self.cfg
        D = cfg.head_dim
        T = ids.numel()
        x = ops.embed_gather(ids, self.embed)
        # decode-sized batches stream the weights through the split-K MFMA kernel; its fp32 slabs
        # are summed by the consumers (RoPE/KV write, RMSNorm) instead of a separate reduction
        max_m = self.STREAM_MAX_M if self.stream else ops.SKINNY_MAX_M
        sk = self.use_skinny and meta.decode and T <= max_m and x.is_cuda
        residual = None
        for li, L in enumerate(self.layers):
            x, residual = self._layer(li, L, x, residual, meta, kv, sk)
        return self._final_norm(x, residual)

    def _final_norm(self, x, residual):
        if x is None:  # the residual stream already holds the last projection (fused prefill add)
            return ops.rmsnorm(residual, self.final_norm, self.cfg.eps)[0]
        return ops.rmsnorm(x, self.final_norm, self.cfg.eps, residual=residual)[0]

    def _layer(self, li: int, L: DecoderLayer, x, residual, meta: AttnMeta, kv: KVCache, sk: bool):
        """One decoder layer: (layer input, residual stream) -> (next layer input, residual stream)."""
        cfg, D, T = self.cfg, self.cfg.head_dim, meta.positions.numel()  # x may be [S, T, H] split-K slabs
        slabs_ok = self.tp_size == 1  # under TP the partial sums go through the all-reduce as bf16
        # prefill (TP 1): the o / down GEMMs add the residual in their epilogue (gemm256 RES, rounded
        # like the separate bf16 add), so the RMSNorms read and write one tensor instead of two each;
        # x is None then: the residual stream already holds the layer input
        fuse = not sk and self.tp_size == 1 and (x if x is not None else residual).is_cuda
        if x is None:
            h, _ = ops.rmsnorm(residual, L.attn_norm, cfg.eps)
        elif residual is None:
            h, _ = ops.rmsnorm(x, L.attn_norm, cfg.eps)
            residual = x
        else:
            h, residual = ops.rmsnorm(x, L.attn_norm, cfg.eps, residual=residual)
        qkv = self._proj(h, L.qkv_w, sk, name="qkv", ws=L.qkv_ws)
        if (not meta.decode and not meta.n_decode and qkv.is_cuda and qkv.dtype == torch.bfloat16
                and ops.kernels.flash_rope_ok(D, kv.block_size)):
            # prefill: the RoPE/KV-write kernel writes only K / V; the attention rotates Q on load
            # straight from the projection (a [T, Hq*D] write and read less per layer)
            ops.rope_kv_write(qkv, meta.positions, self.cos_sin, kv.k[li], kv.v[li], meta.slots, self.hq, self.hkv, D,
                              write_q=False)
            q = qkv[:, :self.hq * D].view(T, self.hq, D)
            a = ops.flash_attention_paged(q, kv.k[li], kv.v[li], meta.block_tables, meta.cu_q, meta.ctx_lens,
                                          meta.max_q, causal=True, rope=(meta.positions, self.cos_sin))
            return self._layer_tail(li, L, a, residual, meta, sk, fuse, slabs_ok, T, D)
        q = ops.rope_kv_write(qkv, meta.positions, self.cos_sin, kv.k[li], kv.v[li], meta.slots, self.hq, self.hkv, D)
        if meta.decode:
            a = ops.paged_decode(q, kv.k[li], kv.v[li], meta.block_tables, meta.ctx_lens, meta.part_size,
                                 meta.workspace, order=meta.order)
        elif meta.n_decode:
            a = self._mixed_attention(q, kv, li, meta)
        else:
            a = ops.flash_attention_paged(q, kv.k[li], kv.v[li], meta.block_tables, meta.cu_q, meta.ctx_lens,
                                          meta.max_q, causal=True)
        return self._layer_tail(li, L, a, residual, meta, sk, fuse, slabs_ok, T, D)

    def _layer_tail(self, li, L, a, residual, meta, sk, fuse, slabs_ok, T, D):
        """o projection, MLP norm, gate_up (+SwiGLU), down: -> (next layer input, residual stream)."""
        cfg = self.cfg
        if fuse:
            residual = ops.gemm_bt(a.view(T, self.hq * D), L.o_w, residual=residual)
            h, _ = ops.rmsnorm(residual, L.mlp_norm, cfg.eps)
        else:
            o = self._all_reduce(self._proj(a.view(T, self.hq * D), L.o_w, sk, slabs_ok, name="o", ws=L.o_ws))
            h, residual = ops.rmsnorm(o, L.mlp_norm, cfg.eps, residual=residual)
        if sk and self.interleaved_mlp and L.gate_up_ws is not None:
            act = ops.stream_gemm(h, L.gate_up_ws, epilogue=ops.EPI_SWIGLU8, nt=True,
                                  cfg=self._stream_cfg("gate_up", T, L.gate_up_ws.shape[0]))
        elif sk and self.interleaved_mlp and "gate_up" in self.skinny_for and T <= ops.SKINNY_MAX_M:
            act = ops.skinny_gemm(h, L.gate_up_w, epilogue=ops.EPI_SWIGLU)
        elif self.interleaved_mlp and h.is_cuda:
            act = ops.gemm_bt(h, L.gate_up_w, epilogue=ops.EPI_SWIGLU)  # SwiGLU in the GEMM epilogue
        else:
            gu = ops.gemm_bt(h, L.gate_up_w) if h.is_cuda else ops.linear(h, L.gate_up_w)
            act = ops.silu_mul(gu, interleaved=self.interleaved_mlp)
        if fuse:
            return None, ops.gemm_bt(act, L.down_w, residual=residual)
        x = self._all_reduce(self._proj(act, L.down_w, sk, slabs_ok, name="down", ws=L.down_ws))
        return x, residual

    def forward_overlapped(self, parts, kv: KVCache) -> torch.Tensor:
        """Prefill of independent sub-batches ``[(ids, meta), ...]`` (disjoint sequences) with each
        sub-batch's layer stack on its own HIP stream, issued layer by layer in lock step.  One
        sub-batch's memory-bound kernels (SiLU-mul, RMSNorm, RoPE/KV write, flash attention) then run
        beside the other's compute-bound hipBLASLt GEMMs instead of after them.  Returns the final
        hidden states of all sub-batches concatenated in order, on the current stream.  Callers
        guarantee no sub-batch reads KV written by another in the same call (prefix blocks are only
        shared once committed after a forward), and TP = 1 (RCCL ordering is per stream)."""
        if len(parts) == 1 or not kv.k.is_cuda:
            return torch.cat([self.forward(ids, meta, kv) for ids, meta in parts])
        main = torch.cuda.current_stream(self.device)
        side = getattr(self, "_side_streams", None)
        if side is None or len(side) < len(parts) - 1:
            side = self._side_streams = [torch.cuda.Stream(self.device) for _ in range(len(parts) - 1)]
        streams = [main] + side[:len(parts) - 1]
        ready = torch.cuda.Event()
        ready.record(main)
        state = []
        for s, (ids, meta) in zip(streams, parts):
            if s is not main:
                s.wait_event(ready)
                # inputs were allocated (and copied in) on the main stream: keep them alive for s
                for t in (ids, meta.positions, meta.slots, meta.block_tables, meta.ctx_lens, meta.cu_q):
                    t.record_stream(s)
            with torch.cuda.stream(s):
                state.append([ops.embed_gather(ids, self.embed), None])
        for li, L in enumerate(self.layers):
            for i, (s, (_, meta)) in enumerate(zip(streams, parts)):
                with torch.cuda.stream(s):
                    state[i] = list(self._layer(li, L, *state[i], meta, kv, False))
        outs = []
        for s, (x, residual) in zip(streams, state):
            with torch.cuda.stream(s):
                outs.append(self._final_norm(x, residual))
        for s, out in zip(streams, outs):
            if s is not main:
                main.wait_stream(s)
                out.record_stream(main)
        return torch.cat(outs)

    @staticmethod
    def _mixed_attention(q, kv: KVCache, li: int, meta: AttnMeta) -> torch.Tensor:
        """Prefill rows through flash attention, decode rows through the split-K paged decode kernel
        (flash's 64-query tiles would be 1/64 full for them and re-read the KV per query head); both
        write disjoint row ranges of one output, so the projections around stay single GEMMs."""
        Tp = q.shape[0] - meta.n_decode
        if not q.is_cuda:
            parts = []
            if Tp:
                parts.append(ops.flash_attention_paged(q[:Tp], kv.k[li], kv.v[li], meta.block_tables, meta.cu_q,
                                                       meta.ctx_lens, meta.max_q, causal=True))
            parts.append(ops.paged_decode(q[Tp:], kv.k[li], kv.v[li], meta.dec_block_tables, meta.dec_ctx_lens,
                                          meta.part_size, meta.workspace))
            return torch.cat(parts)
        a = torch.empty_like(q)
        if Tp:
            ops.flash_attention_paged(q[:Tp], kv.k[li], kv.v[li], meta.block_tables, meta.cu_q, meta.ctx_lens,
                                      meta.max_q, causal=True, out=a[:Tp])
        ops.paged_decode(q[Tp:], kv.k[li], kv.v[li], meta.dec_block_tables, meta.dec_ctx_lens, meta.part_size,
                         meta.workspace, out=a[Tp:])
        return a

    def logits(self, h: torch.Tensor) -> torch.Tensor:
        """[n, H] -> [n, V] logits (bf16; the sampler reads bf16 or fp32).  Up to 256 rows (decode
        steps, prefill last tokens) stream the shuffled LM-head copy through ``stream_gemm``;
        larger batches run the native MFMA GEMM."""
        if not h.is_cuda:
            return ops.linear(h, self.lm_head)
        n = h.shape[0]
        if self.lm_head_ws is not None and n <= self.STREAM_MAX_M:
            cfg = self._stream_cfg("lm_head", n, self.lm_head.shape[0])
            return ops.stream_gemm(h, self.lm_head_ws, cfg=cfg, nt=True)
        if "lm_head" in self.skinny_for and n <= ops.SKINNY_MAX_M and self.lm_head.shape[0] % 64 == 0:
            return ops.skinny_gemm(h, self.lm_head)
        return ops.gemm_bt(h, self.lm_head)
