"""BERT / bge / MiniLM sentence encoder on the native kernels.

Replaces the reference's per-text HF ``AutoModel`` loop (ai/embedders/transformers.py:8-29: batch = 1,
fp32, no truncation, ``last_hidden_state.mean(dim=1)``) with a packed variable-length batch in bf16:

    bert_embed (gather+sum+LN)  ->  L x [ QKV GEMM(+bias)  ->  flash attention (bidirectional, packed)
    ->  O GEMM(+bias+residual)  ->  LN  ->  FFN-up GEMM(+bias+GELU)  ->  FFN-down GEMM(+bias+residual)
    ->  LN ]  ->  mean-pool over all tokens of each sequence (incl. [CLS]/[SEP], like the reference)

No padding tokens are ever computed: sequences are concatenated and delimited by ``cu_seqlens``.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .. import ops
from .configs import EncoderConfig


@dataclass
class EncoderLayer:
    qkv_w: torch.Tensor
    qkv_b: torch.Tensor
    o_w: torch.Tensor
    o_b: torch.Tensor
    ln1_g: torch.Tensor
    ln1_b: torch.Tensor
    i_w: torch.Tensor
    i_b: torch.Tensor
    d_w: torch.Tensor
    d_b: torch.Tensor
    ln2_g: torch.Tensor
    ln2_b: torch.Tensor


class BertEncoder:
    def __init__(self, cfg: EncoderConfig, weights: dict, device: torch.device | str):
        self.cfg = cfg
        self.device = torch.device(device)
        w = {k: v.to(self.device) for k, v in weights.items()}
        self.word = w["word_emb"]
        self.pos = w["pos_emb"]
        self.typ = w["type_emb"]
        self.eln_g = w["emb_ln_g"]
        self.eln_b = w["emb_ln_b"]
        self.layers = [
            EncoderLayer(*(w[f"l{i}.{n}"] for n in ("qkv_w", "qkv_b", "o_w", "o_b", "ln1_g", "ln1_b", "i_w", "i_b",
                                                    "d_w", "d_b", "ln2_g", "ln2_b")))
            for i in range(cfg.layers)
        ]

    @property
    def dtype(self):
        return self.word.dtype

    def forward(self, ids: torch.Tensor, pos_ids: torch.Tensor, cu_seqlens: torch.Tensor, max_seqlen: int):
        """ids / pos_ids int32 [T] packed; cu_seqlens int32 [B+1] -> hidden [T, H]."""
        cfg = self.cfg
        H, nh, D = cfg.hidden, cfg.heads, cfg.head_dim
        T = ids.numel()
        x = ops.bert_embed(ids, pos_ids, None, self.word, self.pos, self.typ, self.eln_g, self.eln_b, cfg.eps)
        for L in self.layers:
            # every projection on the native MFMA GEMM (gemm256 at >= 1024 tokens) with the bias (and
            # the up projection's GELU) in its epilogue; the residual adds too (the bf16 projection
            # plus the residual, rounded: HF's `LayerNorm(dense(x) + input)`), so each LayerNorm reads
            # one tensor
            qkv = ops.linear(x, L.qkv_w, L.qkv_b)
            q = qkv[:, :H].view(T, nh, D)
            k = qkv[:, H:2 * H].view(T, nh, D)
            v = qkv[:, 2 * H:].view(T, nh, D)
            a = ops.flash_attention_packed(q, k, v, cu_seqlens, cu_seqlens, max_seqlen, causal=False)
            h = ops.linear(a.view(T, H), L.o_w, L.o_b, residual=x)
            x = ops.layernorm(h, L.ln1_g, L.ln1_b, cfg.eps)
            f = ops.linear(x, L.i_w, L.i_b, act="gelu")  # bias + GELU(erf) epilogue
            h = ops.linear(f, L.d_w, L.d_b, residual=x)
            x = ops.layernorm(h, L.ln2_g, L.ln2_b, cfg.eps)
        return x

    def encode(self, ids, pos_ids, cu_seqlens, max_seqlen, normalize=None, want_bf16=False):
        """Pooled sentence embeddings fp32 [B, H] (+ bf16 copy)."""
        h = self.forward(ids, pos_ids, cu_seqlens, max_seqlen)
        norm = self.cfg.normalize if normalize is None else normalize
        return ops.mean_pool(h, cu_seqlens, normalize=norm, want_bf16=want_bf16)


def pack_sequences(seqs: list, device, max_len: int | None = None):
    """List of token-id lists -> (ids, pos_ids, cu_seqlens, max_seqlen) int32 tensors on ``device``."""
    import numpy as np

    if max_len:
        seqs = [s[:max_len] for s in seqs]
    lens = np.fromiter((len(s) for s in seqs), dtype=np.int64, count=len(seqs))
    cu = np.zeros(len(seqs) + 1, dtype=np.int32)
    np.cumsum(lens, out=cu[1:])
    total = int(cu[-1])
    ids = np.empty(total, dtype=np.int32)
    pos = np.empty(total, dtype=np.int32)
    for i, s in enumerate(seqs):
        a, b = cu[i], cu[i + 1]
        ids[a:b] = s
        pos[a:b] = np.arange(b - a, dtype=np.int32)
    pin = torch.device(device).type == "cuda"

    def t(a):
        x = torch.from_numpy(a)
        return (x.pin_memory() if pin else x).to(device, non_blocking=True)

    return t(ids), t(pos), t(cu), int(lens.max()) if len(seqs) else 0
