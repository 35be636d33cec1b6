"""Tokenizer facade: a local HF ``tokenizer.json`` when one is provided, else the native hash tokenizer.

The reference uses ``AutoTokenizer.from_pretrained(local_files_only=True)`` (ai/embedders/transformers.py:11,
ai/providers/transformers.py:18).  Here, a directory with ``tokenizer.json`` is loaded through the
``tokenizers`` library (no hub access); otherwise the native C++ ``HashTokenizer`` (csrc/runtime/tokenizer.cpp)
provides the same contract with the model's vocabulary size and special ids.

Chat templates: the reference renders messages as ``"role: content"`` lines (no template;
ai/providers/transformers.py:48).  A checkpoint directory's ``tokenizer_config.json`` template is
available through ``render_chat`` for deployments that opt in (setting ``ENGINE_CHAT_TEMPLATE``):
real instruct checkpoints answer in their trained format.  The Jinja template comes from the local
checkpoint and is rendered in a sandboxed environment (no attribute access to Python internals).
"""
from __future__ import annotations

import os

import numpy as np

from ..models.configs import DecoderConfig, EncoderConfig
from ..ops._lib import native


class Tokenizer:
    def __init__(self, impl, kind: str, hf=None, cls_id=None, sep_id=None, bos_id=None, vocab_size=0,
                 chat_template: dict | None = None):
        self._impl = impl
        self._hf = hf
        self.kind = kind
        self.cls_id, self.sep_id, self.bos_id = cls_id, sep_id, bos_id
        self.vocab_size = vocab_size
        self._chat = chat_template  # {"template", "bos_token", "eos_token"} from tokenizer_config.json
        self._chat_fn = None

    @property
    def has_chat_template(self) -> bool:
        return self._chat is not None

    def render_chat(self, messages: list[dict], add_generation_prompt: bool = True) -> str:
        """The checkpoint's chat template applied to ``messages`` (text; BOS as the template writes it)."""
        if self._chat is None:
            raise ValueError("this tokenizer has no chat template")
        if self._chat_fn is None:
            from jinja2.sandbox import ImmutableSandboxedEnvironment

            env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True)

            def raise_exception(msg):
                raise ValueError(msg)

            env.globals["raise_exception"] = raise_exception
            self._chat_fn = env.from_string(self._chat["template"])
        return self._chat_fn.render(messages=list(messages), add_generation_prompt=add_generation_prompt,
                                    bos_token=self._chat.get("bos_token") or "",
                                    eos_token=self._chat.get("eos_token") or "")

    # ------------------------------------------------------------------ construction
    @classmethod
    def for_encoder(cls, cfg: EncoderConfig, path: str | None = None) -> "Tokenizer":
        hf = _maybe_hf(path)
        if hf is not None:
            return cls(None, "encoder", hf=hf, vocab_size=cfg.vocab_size)
        n = native()
        c = n.TokenizerConfig()
        c.vocab_size = cfg.vocab_size
        c.first_id = 1000 if cfg.vocab_size > 2000 else 200
        c.last_id = cfg.vocab_size
        c.pad_id, c.unk_id, c.cls_id, c.sep_id = 0, 100, 101, 102
        return cls(n.HashTokenizer(c), "encoder", cls_id=101, sep_id=102, vocab_size=cfg.vocab_size)

    @classmethod
    def for_decoder(cls, cfg: DecoderConfig, path: str | None = None) -> "Tokenizer":
        hf = _maybe_hf(path)
        if hf is not None:
            return cls(None, "decoder", hf=hf, bos_id=cfg.bos_id, vocab_size=cfg.vocab_size,
                       chat_template=_chat_template(path))
        n = native()
        c = n.TokenizerConfig()
        c.vocab_size = cfg.vocab_size
        specials_start = min([cfg.bos_id, *cfg.eos_ids])
        c.first_id = 0
        c.last_id = specials_start
        c.pad_id = cfg.eos_ids[0]
        c.unk_id = cfg.eos_ids[0]
        c.cls_id = cfg.bos_id  # BOS
        c.sep_id = -1
        return cls(n.HashTokenizer(c), "decoder", bos_id=cfg.bos_id, vocab_size=cfg.vocab_size)

    @property
    def byte_exact(self) -> bool:
        """Whether every string can be spelled token by token (HF byte-level / SentencePiece
        vocabularies; not the hash tokenizer, whose word tokens carry a leading space)."""
        return self._hf is not None

    # ------------------------------------------------------------------ API
    def encode(self, text: str, add_special: bool = True, max_len: int = 0) -> list[int]:
        if self._hf is not None:
            ids = self._hf.encode(text, add_special_tokens=add_special).ids
            if max_len and len(ids) > max_len:
                ids = ids[: max_len - 1] + ids[-1:] if self.kind == "encoder" else ids[:max_len]
            return ids
        return self._impl.encode(text, add_special, max_len)

    def encode_batch(self, texts: list[str], add_special: bool = True, max_len: int = 0, threads: int = 8):
        """-> (flat int32 ids, int64 offsets[n+1])"""
        if self._hf is not None:
            seqs = [self.encode(t, add_special, max_len) for t in texts]
            offs = np.zeros(len(seqs) + 1, dtype=np.int64)
            np.cumsum([len(s) for s in seqs], out=offs[1:])
            flat = np.fromiter((i for s in seqs for i in s), dtype=np.int32, count=int(offs[-1]))
            return flat, offs
        return self._impl.encode_batch(list(texts), add_special, max_len, threads)

    def decode(self, ids, skip_special: bool = True) -> str:
        ids = [int(i) for i in ids]
        if self._hf is not None:
            return self._hf.decode(ids, skip_special_tokens=skip_special)
        return self._impl.decode(ids, skip_special)

    def count_tokens(self, text: str) -> int:
        return len(self.encode(text, add_special=False))


def _chat_template(path) -> dict | None:
    """``chat_template`` (and the BOS / EOS token strings it references) of a checkpoint directory's
    tokenizer_config.json; a named-template list takes the "default" entry."""
    import json

    f = os.path.join(path, "tokenizer_config.json") if path and os.path.isdir(path) else None
    if not f or not os.path.exists(f):
        return None
    with open(f) as fh:
        c = json.load(fh)
    t = c.get("chat_template")
    if isinstance(t, list):
        t = next((x.get("template") for x in t if x.get("name") == "default"), None)
    if not t:
        return None

    def tok(v):
        return v.get("content") if isinstance(v, dict) else v

    return {"template": t, "bos_token": tok(c.get("bos_token")), "eos_token": tok(c.get("eos_token"))}


def _maybe_hf(path):
    if not path:
        return None
    f = os.path.join(path, "tokenizer.json") if os.path.isdir(path) else path
    if not os.path.exists(f):
        return None
    from tokenizers import Tokenizer as HFTokenizer

    return HFTokenizer.from_file(f)
