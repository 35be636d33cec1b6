"""Model shape presets (public architecture configs) for the encoder and decoder families.

The reference names models by HF hub id (gpu_service/models.py:1-9, settings EMBEDDING_AI_MODEL /
DIALOG_*_AI_MODEL); the engine resolves the same ids (and short aliases) to these presets, builds
random-init weights of the exact shapes (benchmarks) or loads safetensors checkpoints when a local
directory is given.
"""
from __future__ import annotations

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


def encoder_config(name: str, **overrides) -> EncoderConfig:
    k = _key(name)
    if k not in ENCODERS:
        raise KeyError(f"unknown encoder model '{name}' (known: {sorted(ENCODERS)})")
    return replace(ENCODERS[k], **overrides) if overrides else ENCODERS[k]


def decoder_config(name: str, **overrides) -> DecoderConfig:
    k = _key(name)
    if k not in DECODERS:
        raise KeyError(f"unknown decoder model '{name}' (known: {sorted(DECODERS)})")
    return replace(DECODERS[k], **overrides) if overrides else DECODERS[k]


def is_encoder(name: str) -> bool:
    return _key(name) in ENCODERS


def is_decoder(name: str) -> bool:
    return _key(name) in DECODERS
