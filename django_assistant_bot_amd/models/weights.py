"""Weight factories: seeded random init with the real shapes, or HF safetensors checkpoints.

Random init is what the benchmarks use (no network, BASELINE.json "random-init weights"); it is
generated directly on the target device, shard by shard for tensor parallelism, so a 70B TP=8 rank
never materialises more than its own ~17.6 GB.  Checkpoint loading maps HF tensor names to the
engine's fused layouts (QKV concatenated, gate/up stacked or interleaved for the fused SwiGLU GEMM)
and slices the tensor-parallel shard of each projection (Megatron column / row split).
"""
from __future__ import annotations

import glob
import os
import re

import torch

from .configs import DecoderConfig, EncoderConfig

STD = 0.02


def _randn(shape, gen, device, dtype, std=STD):
    t = torch.empty(shape, device=device, dtype=torch.float32)
    t.normal_(0.0, std, generator=gen)
    return t.to(dtype)


def _gen(device, seed):
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    return g


def random_encoder_weights(cfg: EncoderConfig, device="cpu", dtype=torch.bfloat16, seed=0) -> dict:
    device = torch.device(device)
    g = _gen(device, seed)
    H, F = cfg.hidden, cfg.intermediate
    ones = lambda n: torch.ones(n, device=device, dtype=dtype)  # noqa: E731
    zeros = lambda n: torch.zeros(n, device=device, dtype=dtype)  # noqa: E731
    w = {
        "word_emb": _randn((cfg.vocab_size, H), g, device, dtype),
        "pos_emb": _randn((cfg.max_position, H), g, device, dtype),
        "type_emb": _randn((cfg.type_vocab, H), g, device, dtype),
        "emb_ln_g": ones(H),
        "emb_ln_b": zeros(H),
    }
    for i in range(cfg.layers):
        w[f"l{i}.qkv_w"] = _randn((3 * H, H), g, device, dtype)
        w[f"l{i}.qkv_b"] = _randn((3 * H,), g, device, dtype)
        w[f"l{i}.o_w"] = _randn((H, H), g, device, dtype)
        w[f"l{i}.o_b"] = _randn((H,), g, device, dtype)
        w[f"l{i}.ln1_g"] = ones(H)
        w[f"l{i}.ln1_b"] = zeros(H)
        w[f"l{i}.i_w"] = _randn((F, H), g, device, dtype)
        w[f"l{i}.i_b"] = _randn((F,), g, device, dtype)
        w[f"l{i}.d_w"] = _randn((H, F), g, device, dtype)
        w[f"l{i}.d_b"] = _randn((H,), g, device, dtype)
        w[f"l{i}.ln2_g"] = ones(H)
        w[f"l{i}.ln2_b"] = zeros(H)
    return w


def _interleave16(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    Fd, H = gate.shape
    return torch.stack([gate.view(Fd // 16, 16, H), up.view(Fd // 16, 16, H)], dim=1).reshape(2 * Fd, H)


def random_decoder_weights(cfg: DecoderConfig, device="cpu", dtype=torch.bfloat16, seed=0, tp_rank=0, tp_size=1,
                           interleave_mlp=False) -> dict:
    """Shard `tp_rank` of a seeded random-init decoder.  With tp_size == 1 this is the full model."""
    device = torch.device(device)
    H, F, D = cfg.hidden, cfg.intermediate, cfg.head_dim
    assert cfg.heads % tp_size == 0 and cfg.kv_heads % tp_size == 0 and F % tp_size == 0
    hq, hkv, f = cfg.heads // tp_size, cfg.kv_heads // tp_size, F // tp_size
    # replicated tensors (embedding, LM head) are identical on every rank; the layer shards draw from
    # a per-rank stream (tp_size == 1 keeps the single stream)
    g = _gen(device, seed * 1000003)
    w = {
        "embed": _randn((cfg.vocab_size, H), g, device, dtype),
        "final_norm": torch.ones(H, device=device, dtype=dtype),
    }
    if not cfg.tie_embeddings:
        w["lm_head"] = _randn((cfg.vocab_size, H), g, device, dtype)
    if tp_size > 1:
        g = _gen(device, seed * 1000003 + 1 + tp_rank)
    for i in range(cfg.layers):
        w[f"l{i}.attn_norm"] = torch.ones(H, device=device, dtype=dtype)
        w[f"l{i}.qkv_w"] = _randn(((hq + 2 * hkv) * D, H), g, device, dtype)
        w[f"l{i}.o_w"] = _randn((H, hq * D), g, device, dtype)
        w[f"l{i}.mlp_norm"] = torch.ones(H, device=device, dtype=dtype)
        gate = _randn((f, H), g, device, dtype)
        up = _randn((f, H), g, device, dtype)
        w[f"l{i}.gate_up_w"] = _interleave16(gate, up) if interleave_mlp else torch.cat([gate, up], 0)
        del gate, up
        w[f"l{i}.down_w"] = _randn((H, f), g, device, dtype)
    return w


def shard_decoder_weights(full: dict, cfg: DecoderConfig, tp_rank: int, tp_size: int, interleave_mlp=False) -> dict:
    """Megatron split of a full (stacked gate|up) decoder state: QKV / gate-up by output rows
    (column parallel), O / down by input columns (row parallel)."""
    H, F, D = cfg.hidden, cfg.intermediate, cfg.head_dim
    hq, hkv, f = cfg.heads // tp_size, cfg.kv_heads // tp_size, F // tp_size
    out = {k: v for k, v in full.items() if not re.match(r"l\d+\.", k)}  # embed, final_norm, lm_head
    for i in range(cfg.layers):
        qkv = full[f"l{i}.qkv_w"]
        q = qkv[: cfg.heads * D].view(cfg.heads, D, H)[tp_rank * hq:(tp_rank + 1) * hq].reshape(-1, H)
        k = qkv[cfg.heads * D:(cfg.heads + cfg.kv_heads) * D].view(cfg.kv_heads, D, H)
        v = qkv[(cfg.heads + cfg.kv_heads) * D:].view(cfg.kv_heads, D, H)
        k = k[tp_rank * hkv:(tp_rank + 1) * hkv].reshape(-1, H)
        v = v[tp_rank * hkv:(tp_rank + 1) * hkv].reshape(-1, H)
        out[f"l{i}.qkv_w"] = torch.cat([q, k, v], 0).contiguous()
        out[f"l{i}.o_w"] = full[f"l{i}.o_w"][:, tp_rank * hq * D:(tp_rank + 1) * hq * D].contiguous()
        gu = full[f"l{i}.gate_up_w"]
        gate = gu[:F][tp_rank * f:(tp_rank + 1) * f]
        up = gu[F:][tp_rank * f:(tp_rank + 1) * f]
        out[f"l{i}.gate_up_w"] = (_interleave16(gate, up) if interleave_mlp else torch.cat([gate, up], 0)).contiguous()
        out[f"l{i}.down_w"] = full[f"l{i}.down_w"][:, tp_rank * f:(tp_rank + 1) * f].contiguous()
        out[f"l{i}.attn_norm"] = full[f"l{i}.attn_norm"]
        out[f"l{i}.mlp_norm"] = full[f"l{i}.mlp_norm"]
    return out


# ------------------------------------------------------------------------------------------------
# HF checkpoints (safetensors only: nothing executable is ever loaded)


def _read_safetensors(path: str) -> dict:
    from safetensors.torch import load_file

    files = sorted(glob.glob(os.path.join(path, "*.safetensors"))) if os.path.isdir(path) else [path]
    if not files:
        raise FileNotFoundError(f"no .safetensors files under {path}")
    state = {}
    for f in files:
        state.update(load_file(f))
    return state


def load_encoder_checkpoint(path: str, cfg: EncoderConfig, dtype=torch.bfloat16) -> dict:
    st = _read_safetensors(path)
    pre = "bert." if any(k.startswith("bert.") for k in st) else ""
    get = lambda k: st[pre + k].to(dtype)  # noqa: E731
    w = {
        "word_emb": get("embeddings.word_embeddings.weight"),
        "pos_emb": get("embeddings.position_embeddings.weight"),
        "type_emb": get("embeddings.token_type_embeddings.weight"),
        "emb_ln_g": get("embeddings.LayerNorm.weight"),
        "emb_ln_b": get("embeddings.LayerNorm.bias"),
    }
    for i in range(cfg.layers):
        p = f"encoder.layer.{i}."
        w[f"l{i}.qkv_w"] = torch.cat([get(p + f"attention.self.{n}.weight") for n in ("query", "key", "value")], 0)
        w[f"l{i}.qkv_b"] = torch.cat([get(p + f"attention.self.{n}.bias") for n in ("query", "key", "value")], 0)
        w[f"l{i}.o_w"] = get(p + "attention.output.dense.weight")
        w[f"l{i}.o_b"] = get(p + "attention.output.dense.bias")
        w[f"l{i}.ln1_g"] = get(p + "attention.output.LayerNorm.weight")
        w[f"l{i}.ln1_b"] = get(p + "attention.output.LayerNorm.bias")
        w[f"l{i}.i_w"] = get(p + "intermediate.dense.weight")
        w[f"l{i}.i_b"] = get(p + "intermediate.dense.bias")
        w[f"l{i}.d_w"] = get(p + "output.dense.weight")
        w[f"l{i}.d_b"] = get(p + "output.dense.bias")
        w[f"l{i}.ln2_g"] = get(p + "output.LayerNorm.weight")
        w[f"l{i}.ln2_b"] = get(p + "output.LayerNorm.bias")
    return {k: v.contiguous() for k, v in w.items()}


def load_decoder_checkpoint(path: str, cfg: DecoderConfig, dtype=torch.bfloat16, tp_rank=0, tp_size=1,
                            interleave_mlp=False) -> dict:
    st = _read_safetensors(path)
    get = lambda k: st[k].to(dtype)  # noqa: E731
    full = {"embed": get("model.embed_tokens.weight"), "final_norm": get("model.norm.weight")}
    if not cfg.tie_embeddings:
        full["lm_head"] = get("lm_head.weight")
    for i in range(cfg.layers):
        p = f"model.layers.{i}."
        full[f"l{i}.attn_norm"] = get(p + "input_layernorm.weight")
        full[f"l{i}.qkv_w"] = torch.cat([get(p + f"self_attn.{n}_proj.weight") for n in ("q", "k", "v")], 0)
        full[f"l{i}.o_w"] = get(p + "self_attn.o_proj.weight")
        full[f"l{i}.mlp_norm"] = get(p + "post_attention_layernorm.weight")
        full[f"l{i}.gate_up_w"] = torch.cat([get(p + "mlp.gate_proj.weight"), get(p + "mlp.up_proj.weight")], 0)
        full[f"l{i}.down_w"] = get(p + "mlp.down_proj.weight")
    return shard_decoder_weights(full, cfg, tp_rank, tp_size, interleave_mlp)
