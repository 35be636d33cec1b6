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
        inv = ref.llama3_inv_freq(cfg.head_dim, cfg.rope_theta, cfg.rope_scaling)
        self.cos_sin = ref.rope_cos_sin(inv, cfg.max_position).to(self.device)

    @property
    def dtype(self):
        return self.embed.dtype

    def _all_reduce(self, x):
        if self.tp_size > 1:
            import torch.distributed as dist

            dist.all_reduce(x, group=self.tp_group)
        return x

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: KVCache) -> torch.Tensor:
        """ids int32 [T] -> final hidden states [T, H] (after the last RMSNorm)."""
        cfg = self.cfg
        D = cfg.head_dim
        T = ids.numel()
        x = ops.embed_gather(ids, self.embed)
        residual = None
        for li, L in enumerate(self.layers):
            if residual is None:
                h, _ = ops.rmsnorm(x, L.attn_norm, cfg.eps)
                residual = x
            else:
                h, residual = ops.rmsnorm(x, L.attn_norm, cfg.eps, residual=residual)
            qkv = ops.linear(h, L.qkv_w)
            q = ops.rope_kv_write(qkv, meta.positions, self.cos_sin, kv.k[li], kv.v[li], meta.slots, self.hq, self.hkv,
                                  D)
            if meta.decode:
                a = ops.paged_decode(q, kv.k[li], kv.v[li], meta.block_tables, meta.ctx_lens, meta.part_size,
                                     meta.workspace)
            else:
                a = ops.flash_attention_paged(q, kv.k[li], kv.v[li], meta.block_tables, meta.cu_q, meta.ctx_lens,
                                              meta.max_q, causal=True)
            o = self._all_reduce(ops.linear(a.view(T, self.hq * D), L.o_w))
            h, residual = ops.rmsnorm(o, L.mlp_norm, cfg.eps, residual=residual)
            if self.interleaved_mlp:
                act = ops.linear(h, L.gate_up_w, act="swiglu")
            else:
                act = ops.silu_mul(ops.linear(h, L.gate_up_w))
            x = self._all_reduce(ops.linear(act, L.down_w))
        out, _ = ops.rmsnorm(x, self.final_norm, cfg.eps, residual=residual)
        return out

    def logits(self, h: torch.Tensor) -> torch.Tensor:
        """[n, H] -> [n, V] logits (bf16 GEMM; the sampler reads bf16 or fp32)."""
        return ops.linear(h, self.lm_head)
