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


MLP_GROUP = 8  # gate|up row groups of the fused SwiGLU GEMMs (EPI_SWIGLU8: any 16-row tile holds pairs)


def _mlp_group(interleave_mlp) -> int:
    """``interleave_mlp``: False / 0 = stacked [gate; up], True = the engine's 8-row groups, or an
    explicit group size (8 / 16)."""
    if interleave_mlp is True:
        return MLP_GROUP
    return int(interleave_mlp or 0)


def _gate_up(gate: torch.Tensor, up: torch.Tensor, interleave_mlp) -> torch.Tensor:
    grp = _mlp_group(interleave_mlp)
    if not grp:
        return torch.cat([gate, up], 0)
    Fd, H = gate.shape
    return torch.stack([gate.reshape(Fd // grp, grp, H), up.reshape(Fd // grp, grp, H)], dim=1).reshape(2 * Fd, H)


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
        w[f"l{i}.gate_up_w"] = _gate_up(gate, up, interleave_mlp)
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
        out[f"l{i}.gate_up_w"] = _gate_up(gate, up, interleave_mlp).contiguous()
        out[f"l{i}.down_w"] = full[f"l{i}.down_w"][:, tp_rank * f:(tp_rank + 1) * f].contiguous()
        out[f"l{i}.attn_norm"] = full[f"l{i}.attn_norm"]
        out[f"l{i}.mlp_norm"] = full[f"l{i}.mlp_norm"]
    return out


# ------------------------------------------------------------------------------------------------
# HF checkpoints (safetensors only: nothing executable is ever loaded)


class SafetensorsDir:
    """Lazy reader over the ``*.safetensors`` files of a checkpoint (``safe_open``: memory-mapped,
    nothing executable).  ``get`` materialises a whole tensor, ``rows`` / ``cols`` only a slice, so
    a tensor-parallel rank reads about 1/tp of every sharded projection.  ``bytes_read`` counts the
    bytes materialised (tests / logs)."""

    def __init__(self, path: str):
        from safetensors import safe_open

        files = sorted(glob.glob(os.path.join(path, "*.safetensors"))) if os.path.isdir(path) else [path]
        if not files:
            raise FileNotFoundError(f"no .safetensors files under {path}")
        self._handles = [safe_open(f, framework="pt") for f in files]
        self._where = {k: h for h in self._handles for k in h.keys()}
        self.bytes_read = 0

    def keys(self):
        return self._where.keys()

    def __contains__(self, name):
        return name in self._where

    def _count(self, t):
        self.bytes_read += t.numel() * t.element_size()
        return t

    def get(self, name):
        return self._count(self._where[name].get_tensor(name))

    def rows(self, name, a: int, b: int):
        return self._count(self._where[name].get_slice(name)[a:b])

    def cols(self, name, a: int, b: int):
        return self._count(self._where[name].get_slice(name)[:, a:b])


def _read_safetensors(path: str) -> dict:
    st = SafetensorsDir(path)
    return {k: st.get(k) for k in st.keys()}


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
                            interleave_mlp=False, reader: SafetensorsDir | None = None) -> dict:
    """The rank's tensor-parallel shard of an HF Llama checkpoint, read slice by slice: q / k / v /
    gate / up by output rows (column parallel), o / down by input columns (row parallel), so a rank
    of a 70B TP-8 group materialises ~1/8 of every projection (~17.5 GB) instead of the whole
    140 GB state.  Replicated tensors (embedding, LM head, norms) are read whole.  Same result as
    ``shard_decoder_weights`` of the full state (tests/test_models_cpu.py)."""
    st = reader or SafetensorsDir(path)
    H, F, D = cfg.hidden, cfg.intermediate, cfg.head_dim
    hq, hkv, f = cfg.heads // tp_size, cfg.kv_heads // tp_size, F // tp_size
    cast = lambda t: t.to(dtype).contiguous()  # noqa: E731
    w = {"embed": cast(st.get("model.embed_tokens.weight")), "final_norm": cast(st.get("model.norm.weight"))}
    if not cfg.tie_embeddings:
        w["lm_head"] = cast(st.get("lm_head.weight"))
    r = tp_rank
    for i in range(cfg.layers):
        p = f"model.layers.{i}."
        w[f"l{i}.attn_norm"] = cast(st.get(p + "input_layernorm.weight"))
        w[f"l{i}.mlp_norm"] = cast(st.get(p + "post_attention_layernorm.weight"))
        q = st.rows(p + "self_attn.q_proj.weight", r * hq * D, (r + 1) * hq * D)
        k = st.rows(p + "self_attn.k_proj.weight", r * hkv * D, (r + 1) * hkv * D)
        v = st.rows(p + "self_attn.v_proj.weight", r * hkv * D, (r + 1) * hkv * D)
        w[f"l{i}.qkv_w"] = cast(torch.cat([q, k, v], 0))
        w[f"l{i}.o_w"] = cast(st.cols(p + "self_attn.o_proj.weight", r * hq * D, (r + 1) * hq * D))
        gate = st.rows(p + "mlp.gate_proj.weight", r * f, (r + 1) * f).to(dtype)
        up = st.rows(p + "mlp.up_proj.weight", r * f, (r + 1) * f).to(dtype)
        w[f"l{i}.gate_up_w"] = _gate_up(gate, up, interleave_mlp).contiguous()
        w[f"l{i}.down_w"] = cast(st.cols(p + "mlp.down_proj.weight", r * f, (r + 1) * f))
    return w
