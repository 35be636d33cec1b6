"""Model shape presets (public architecture configs) for the encoder and decoder families.

The reference names models by HF hub id (gpu_service/models.py:1-9, settings EMBEDDING_AI_MODEL /
DIALOG_*_AI_MODEL); the engine resolves the same ids (and short aliases) to these presets, builds
random-init weights of the exact shapes (benchmarks) or loads safetensors checkpoints when a local
directory is given.
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass, field, replace


@dataclass(frozen=True)
class EncoderConfig:
    name: str
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_position: int = 512
    type_vocab: int = 2
    eps: float = 1e-12
    normalize: bool = False  # reference mean-pools and does NOT L2-normalise (embedders/transformers.py:25)

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    def to_dict(self):
        return asdict(self)


@dataclass(frozen=True)
class DecoderConfig:
    name: str
    vocab_size: int = 128256
    hidden: int = 4096
    layers: int = 32
    heads: int = 32
    kv_heads: int = 8
    intermediate: int = 14336
    rope_theta: float = 500000.0
    rope_scaling: dict | None = field(default_factory=lambda: {
        "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0, "original_max_position_embeddings": 8192})
    eps: float = 1e-5
    max_position: int = 8192
    bos_id: int = 128000
    eos_ids: tuple = (128001, 128009)
    tie_embeddings: bool = False

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    def to_dict(self):
        return asdict(self)

    def params(self) -> int:
        H, F, V, L = self.hidden, self.intermediate, self.vocab_size, self.layers
        D = self.head_dim
        attn = H * (self.heads * D) + 2 * H * (self.kv_heads * D) + (self.heads * D) * H
        mlp = 3 * H * F
        emb = V * H * (1 if self.tie_embeddings else 2)
        return L * (attn + mlp + 2 * H) + emb + H


ENCODERS = {
    "bge-base-en": EncoderConfig("bge-base-en"),
    "bge-large-en": EncoderConfig("bge-large-en", hidden=1024, layers=24, heads=16, intermediate=4096),
    "all-minilm-l6": EncoderConfig("all-minilm-l6", hidden=384, layers=6, heads=12, intermediate=1536),
    "rubert-base": EncoderConfig("rubert-base", vocab_size=120138),
    "tiny-bert": EncoderConfig("tiny-bert", vocab_size=2048, hidden=128, layers=2, heads=2, intermediate=256,
                               max_position=128),
}

DECODERS = {
    "llama-3-8b": DecoderConfig("llama-3-8b"),
    "llama-3-70b": DecoderConfig("llama-3-70b", hidden=8192, layers=80, heads=64, kv_heads=8, intermediate=28672),
    "llama-3.2-1b": DecoderConfig("llama-3.2-1b", hidden=2048, layers=16, heads=32, kv_heads=8, intermediate=8192,
                                  tie_embeddings=True,
                                  rope_scaling={"factor": 32.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                                "original_max_position_embeddings": 8192}),
    "tiny-llama": DecoderConfig("tiny-llama", vocab_size=1024, hidden=256, layers=2, heads=4, kv_heads=2,
                                intermediate=512, max_position=2048, bos_id=1000, eos_ids=(1001,), rope_scaling=None,
                                rope_theta=10000.0),
    # the Llama-3-70B head layout (64 query heads over 8 KV heads) at toy width: at TP=8 every rank
    # holds exactly one KV head and 8 query heads, like 70B on 8 GPUs (CPU multi-rank tests)
    "tiny-llama-70b-layout": DecoderConfig("tiny-llama-70b-layout", vocab_size=1024, hidden=1024, layers=2, heads=64,
                                           kv_heads=8, intermediate=1024, max_position=2048, bos_id=1000,
                                           eos_ids=(1001,), rope_scaling=None, rope_theta=10000.0),
    # Llama-3-70B's real attention layout (hidden 8192, 64 / 8 heads of D = 128) at 2 layers with a
    # toy vocabulary and MLP: TP=8 ranks run the D = 128 prefill / decode attention kernels with 8
    # query heads over 1 KV head and all-reduce 70B-sized rows (B x 8192)
    "tiny-llama-70b-d128": DecoderConfig("tiny-llama-70b-d128", vocab_size=1024, hidden=8192, layers=2, heads=64,
                                         kv_heads=8, intermediate=2048, max_position=2048, bos_id=1000,
                                         eos_ids=(1001,), rope_scaling=None, rope_theta=10000.0),
}

_ALIASES = {
    "baai/bge-base-en": "bge-base-en", "baai/bge-base-en-v1.5": "bge-base-en", "bge-base": "bge-base-en",
    "baai/bge-large-en": "bge-large-en", "baai/bge-large-en-v1.5": "bge-large-en", "bge-large": "bge-large-en",
    "sentence-transformers/all-minilm-l6-v2": "all-minilm-l6", "all-minilm-l6-v2": "all-minilm-l6",
    "sberbank-ai/rubert-base": "rubert-base", "ai-forever/rubert-base": "rubert-base",
    "meta-llama/meta-llama-3-8b": "llama-3-8b", "meta-llama/meta-llama-3-8b-instruct": "llama-3-8b",
    "meta-llama/llama-3.1-8b-instruct": "llama-3-8b", "llama3": "llama-3-8b", "llama3:8b": "llama-3-8b",
    "llama-3.1-8b": "llama-3-8b",
    "meta-llama/meta-llama-3-70b-instruct": "llama-3-70b", "llama3:70b": "llama-3-70b", "llama-3.1-70b": "llama-3-70b",
    "meta-llama/llama-3.2-1b-instruct": "llama-3.2-1b",
}


def _key(name: str) -> str:
    k = name.strip().lower()
    return _ALIASES.get(k, k)


# ------------------------------------------------------------------ local HF checkpoint directories
# A model name may also be a local HF directory (config.json + *.safetensors [+ tokenizer.json]), as
# the reference's TransformersEmbedder / TransformersProvider accept (ai/embedders/transformers.py:13,
# ai/providers/transformers.py:18-20: ``from_pretrained(model_name)``).  The architecture comes from
# config.json; only the families the native kernels implement are accepted.

def checkpoint_dir(name) -> str | None:
    """``name`` if it is a local directory with a config.json, else None."""
    if isinstance(name, str) and os.path.isfile(os.path.join(name, "config.json")):
        return name
    return None


def _hf(path: str) -> dict:
    with open(os.path.join(path, "config.json")) as f:
        return json.load(f)


def _label(path: str) -> str:
    return os.path.basename(os.path.normpath(path)).lower()


def encoder_config_from_hf(path: str) -> EncoderConfig:
    c = _hf(path)
    if c.get("model_type") != "bert":
        raise ValueError(f"{path}: model_type {c.get('model_type')!r} is not a BERT encoder")
    if c.get("hidden_act", "gelu") != "gelu" or c.get("position_embedding_type", "absolute") != "absolute":
        raise ValueError(f"{path}: only erf-GELU BERT encoders with absolute positions are supported")
    return EncoderConfig(_label(path), vocab_size=c["vocab_size"], hidden=c["hidden_size"],
                         layers=c["num_hidden_layers"], heads=c["num_attention_heads"],
                         intermediate=c["intermediate_size"], max_position=c.get("max_position_embeddings", 512),
                         type_vocab=c.get("type_vocab_size", 2), eps=c.get("layer_norm_eps", 1e-12))


def decoder_config_from_hf(path: str) -> DecoderConfig:
    c = _hf(path)
    if c.get("model_type") != "llama":
        raise ValueError(f"{path}: model_type {c.get('model_type')!r} is not a Llama decoder")
    if c.get("hidden_act", "silu") != "silu" or c.get("attention_bias") or c.get("mlp_bias"):
        raise ValueError(f"{path}: only bias-free SiLU Llama decoders are supported")
    heads = c["num_attention_heads"]
    if c.get("head_dim", c["hidden_size"] // heads) * heads != c["hidden_size"]:
        raise ValueError(f"{path}: head_dim x heads must equal hidden_size")
    # transformers 4.x: rope_theta + rope_scaling; 5.x: rope_parameters (theta and scaling together)
    rp = c.get("rope_parameters") or {}
    theta = c.get("rope_theta", rp.get("rope_theta", 10000.0))
    rs = c.get("rope_scaling") or (rp if rp.get("rope_type") not in (None, "default") else None)
    if rs is not None:
        kind = rs.get("rope_type", rs.get("type"))
        if kind == "default":
            rs = None
        elif kind != "llama3":
            raise ValueError(f"{path}: rope_scaling type {kind!r} is not supported (llama3 or none)")
        else:
            rs = {k: float(rs[k]) if k != "original_max_position_embeddings" else int(rs[k])
                  for k in ("factor", "low_freq_factor", "high_freq_factor", "original_max_position_embeddings")}
    eos = c.get("eos_token_id")
    eos = tuple(eos) if isinstance(eos, (list, tuple)) else ((eos,) if eos is not None else ())
    return DecoderConfig(_label(path), vocab_size=c["vocab_size"], hidden=c["hidden_size"],
                         layers=c["num_hidden_layers"], heads=heads,
                         kv_heads=c.get("num_key_value_heads") or heads, intermediate=c["intermediate_size"],
                         rope_theta=float(theta), rope_scaling=rs,
                         eps=float(c.get("rms_norm_eps", 1e-6)), max_position=c.get("max_position_embeddings", 8192),
                         bos_id=c.get("bos_token_id", 1) if c.get("bos_token_id") is not None else 1,
                         eos_ids=eos or (2,), tie_embeddings=bool(c.get("tie_word_embeddings", False)))


def encoder_config(name: str, **overrides) -> EncoderConfig:
    if checkpoint_dir(name):
        cfg = encoder_config_from_hf(name)
        return replace(cfg, **overrides) if overrides else cfg
    k = _key(name)
    if k not in ENCODERS:
        raise KeyError(f"unknown encoder model '{name}' (known: {sorted(ENCODERS)}, or a local HF directory)")
    return replace(ENCODERS[k], **overrides) if overrides else ENCODERS[k]


def decoder_config(name: str, **overrides) -> DecoderConfig:
    if checkpoint_dir(name):
        cfg = decoder_config_from_hf(name)
        return replace(cfg, **overrides) if overrides else cfg
    k = _key(name)
    if k not in DECODERS:
        raise KeyError(f"unknown decoder model '{name}' (known: {sorted(DECODERS)}, or a local HF directory)")
    return replace(DECODERS[k], **overrides) if overrides else DECODERS[k]


def is_encoder(name: str) -> bool:
    d = checkpoint_dir(name)
    return _hf(d).get("model_type") == "bert" if d else _key(name) in ENCODERS


def is_decoder(name: str) -> bool:
    d = checkpoint_dir(name)
    return _hf(d).get("model_type") == "llama" if d else _key(name) in DECODERS
