"""JSON-constrained decoding: the vocabulary side (token byte strings for the native automaton).

The reference gets JSON from its generators by asking for it and retrying until ``json.loads``
succeeds (up to 5 generations: /root/reference/assistant/bot/services/context_service/steps/
classify.py:41-45, choose_known_question.py:45-50).  Here a request with
``SamplingParams(json_mode=True)`` carries a native ``JsonMatcher`` (csrc/runtime/json_grammar.cpp):
before each sampling step the engine asks it for the allowed-token bitmask, the ``mask_logits``
kernel sets every other logit to -inf, and the sampled token advances the automaton.  The output is
one JSON object, closed within ``max_new_tokens``; generation stops as soon as it is complete.

Token byte strings:
  * HF byte-level BPE (Llama-3, GPT-2 style ``tokenizer.json``): the token string's characters map
    back to bytes through the GPT-2 byte <-> unicode table;
  * SentencePiece-style vocabularies: ``▁`` is a space, ``<0xNN>`` a raw byte;
  * the native hash tokenizer: ``HashTokenizer.token_texts`` (what each id adds to ``decode``);
  * special / added tokens contribute nothing and are never allowed (EOS once the object is done).
"""
from __future__ import annotations

import json
import threading

from ..ops._lib import native

_JSON_PUNCT = '{ } [ ] : , " \\ - + . e E 0 1 2 3 4 5 6 7 8 9 true false null'
_lock = threading.Lock()


def _byte_decoder() -> dict:
    """Inverse of GPT-2's bytes_to_unicode: printable bytes map to themselves, the rest to 256+."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("\xa1"), ord("\xac") + 1)) + \
        list(range(ord("\xae"), ord("\xff") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {chr(c): b for b, c in zip(bs, cs)}


def hf_token_bytes(hf, vocab_size: int) -> list[bytes]:
    """Byte string of every id of a ``tokenizers.Tokenizer`` (b"" for special / added tokens)."""
    spec = json.loads(hf.to_str())
    dec = spec.get("decoder") or {}
    kinds = {dec.get("type")} | {d.get("type") for d in dec.get("decoders", []) or []}
    byte_level = "ByteLevel" in kinds
    special = {int(a["id"]) for a in spec.get("added_tokens", []) if a.get("special", True)}
    out = [b""] * vocab_size
    bdec = _byte_decoder() if byte_level else None
    for tok, i in hf.get_vocab(with_added_tokens=True).items():
        if i >= vocab_size or i in special:
            continue
        if byte_level:
            try:
                out[i] = bytes(bdec[c] for c in tok)
            except KeyError:  # an added non-byte-level token
                out[i] = tok.encode("utf-8")
        elif len(tok) == 6 and tok.startswith("<0x") and tok.endswith(">"):
            out[i] = bytes([int(tok[3:5], 16)])
        else:
            out[i] = tok.replace("▁", " ").encode("utf-8")
    return out


def vocab_for(tokenizer, eos_ids) -> "native().JsonVocab":
    """The (cached) native JSON vocabulary of an engine ``Tokenizer``."""
    with _lock:
        v = getattr(tokenizer, "_json_vocab", None)
        if v is not None:
            return v
        V = tokenizer.vocab_size
        if tokenizer._hf is not None:
            toks = hf_token_bytes(tokenizer._hf, V)
        else:
            tokenizer.encode(_JSON_PUNCT, add_special=False)  # JSON punctuation decodes as itself
            toks = list(tokenizer._impl.token_texts())
        v = native().JsonVocab(toks, [int(e) for e in eos_ids])
        tokenizer._json_vocab = v
        return v


def matcher_for(tokenizer, eos_ids, max_depth: int = 24, max_ws: int = 8):
    return native().JsonMatcher(vocab_for(tokenizer, eos_ids), max_depth, max_ws)
