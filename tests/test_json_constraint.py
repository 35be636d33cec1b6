"""JSON-constrained decoding (csrc/runtime/json_grammar.cpp, engine/json_constraint.py).

The reference retries its JSON steps until ``json.loads`` succeeds (up to 5 generations,
/root/reference/assistant/bot/services/context_service/steps/classify.py:41-45); here the sampler
is masked to the grammar so one generation is valid.  Checked: the automaton against Python's json
parser (accept / reject, completions of every prefix), the per-step token masks against a brute
force over the vocabulary (budget included), and end-to-end engine generations that always parse.
"""
import json
import random

import numpy as np
import pytest

from django_assistant_bot_amd.ops import native


def _rand_value(rng, depth=0):
    k = rng.randrange(8 if depth < 4 else 5)
    if k == 0:
        return rng.randrange(-10**6, 10**6)
    if k == 1:
        return rng.choice([0.5, -1.25e-7, 3.0e21, 1e-300, -0.0])
    if k == 2:
        return "".join(rng.choice(["a", "б", "\"", "\\", "\n", "\t", "/", "é", "😀", " ", "\u0001", "x"])
                       for _ in range(rng.randrange(6)))
    if k == 3:
        return rng.choice([True, False, None])
    if k == 4:
        return ""
    if k == 5:
        return [_rand_value(rng, depth + 1) for _ in range(rng.randrange(4))]
    return {"k%d%s" % (i, rng.choice(["", "é", '"'])): _rand_value(rng, depth + 1) for i in range(rng.randrange(4))}


def _docs(n=150, seed=0):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        obj = {f"key{j}": _rand_value(rng) for j in range(rng.randrange(1, 4))}
        indent = [None, 0, 2][i % 3]
        out.append(json.dumps(obj, indent=indent, ensure_ascii=bool(i % 2)).encode())
    out += [b"{}", b' { "a" : [ ] , "b":{}}\n', b'{"x":-0.5e+10,"y":[true,false,null,0,1e5,2E-3]}']
    return out


def _byte_vocab():
    n = native()
    toks = [bytes([b]) for b in range(256)] + [b""]  # id 256: EOS
    return n.JsonVocab(toks, [256])


def test_automaton_accepts_valid_json_and_completes_every_prefix():
    n = native()
    v = _byte_vocab()
    for doc in _docs():
        assert n.json_accepts(doc, True), doc
        m = n.JsonMatcher(v, 64, 255)
        for i, b in enumerate(doc):
            assert m.advance(b), (doc, i)
            if i % 3 == 0 or i == len(doc) - 1:
                comp = m.completion()
                assert len(comp) == m.completion_len()
                got = json.loads((doc[:i + 1] + comp).decode("utf-8", errors="replace"))  # a cut character
                assert isinstance(got, dict)
        assert m.done() and m.completion() == b""


@pytest.mark.parametrize("seed", range(4))
def test_automaton_rejects_what_python_rejects(seed):
    """Byte mutations of valid documents: complete acceptance == json.loads gives a dict (Python's
    NaN / Infinity extensions excluded); a rejected document's failing prefix is never accepted."""
    n = native()
    rng = random.Random(seed)
    docs = _docs(60, seed + 10)
    alphabet = b'{}[]:,"\\-+.eE0123456789tfnulrsa \n\x01'
    checked = 0
    for doc in docs:
        for _ in range(12):
            b = bytearray(doc)
            for _ in range(rng.randrange(1, 3)):
                op = rng.randrange(3)
                pos = rng.randrange(len(b) + 1)
                if op == 0 and len(b) > 1:
                    del b[min(pos, len(b) - 1)]
                elif op == 1:
                    b.insert(pos, rng.choice(alphabet))
                elif len(b):
                    b[min(pos, len(b) - 1)] = rng.choice(alphabet)
            data = bytes(b)
            if b"NaN" in data or b"Infinity" in data:
                continue
            try:
                ok = isinstance(json.loads(data.decode("utf-8")), dict)
            except (ValueError, UnicodeDecodeError):
                ok = False
            if ok:  # Python accepts some documents our object-only top level does not: none here
                assert n.json_accepts(data, True), data
            else:
                # utf-8 validity is not the automaton's business (byte tokens may split characters)
                try:
                    data.decode("utf-8")
                except UnicodeDecodeError:
                    continue
                assert not n.json_accepts(data, True), data
            checked += 1
    assert checked > 300


def _brute_mask(toks, prefix_ids, remaining, max_depth=24, max_ws=8):
    n = native()
    v = n.JsonVocab(toks, [len(toks) - 1])
    allowed = set()
    for t in range(len(toks)):
        m = n.JsonMatcher(v, max_depth, max_ws)
        for p in prefix_ids:
            assert m.advance(p)
        base = m.completion_len()
        if t == len(toks) - 1:
            if m.done():
                allowed.add(t)
            continue
        if toks[t] and m.advance(t) and m.completion_len() <= min(max(remaining - 1, 0), base + 64):
            allowed.add(t)
    return allowed


def _mask_set(m, V, remaining):
    W = -(-V // 32)
    buf = np.zeros(W, dtype=np.int32)
    cnt = m.fill_mask(remaining, buf.ctypes.data)
    bits = np.unpackbits(buf.view(np.uint8), bitorder="little")[:V]
    s = set(np.nonzero(bits)[0].tolist())
    assert cnt == len(s)
    return s


def test_masks_match_brute_force_with_budget():
    """A small vocabulary with multi-byte tokens; every completion byte has a single-byte token (as
    in byte-level vocabularies), so the budget rule can always close the object."""
    toks = [b"{", b"}", b"[", b"]", b":", b",", b'"', b"a", b"1", b"-", b".", b"e", b" ", b"\n", b"true", b"nul",
            b"l", b"u", b'{"', b'":', b'"}', b"}}", b'"a"', b' "b"', b"12", b"0", b"\\", b"n", b"u00e9", b"\xd0\xb1",
            b'}\n', b'[{"', b"]}", b"tr", b"ue", b"", b"<eos>"]
    toks[-1] = b""  # EOS has no bytes
    n = native()
    v = n.JsonVocab(toks, [len(toks) - 1])
    rng = random.Random(3)
    for trial in range(40):
        m = n.JsonMatcher(v, 24, 8)
        prefix = []
        budget = rng.randrange(2, 14)
        for step in range(budget):
            remaining = budget - step
            got = _mask_set(m, len(toks), remaining)
            assert got == _brute_mask(toks, prefix, remaining), (trial, step, prefix)
            if m.done():
                break
            t = rng.choice(sorted(got))
            assert m.advance(t)
            prefix.append(t)
        # the budget closes the object in time
        assert m.done(), [toks[t] for t in prefix]


def test_mask_falls_back_when_the_budget_cannot_be_met():
    toks = [b"{", b"}", b'"', b"a", b""]
    n = native()
    m = n.JsonMatcher(n.JsonVocab(toks, [4]), 24, 8)
    assert _mask_set(m, 5, 1) == {0}  # "{}" needs 2 tokens: grammar-only mask
    m.advance(0)
    assert _mask_set(m, 5, 1) == {1}


def _engine(**kw):
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine

    return LLMEngine("tiny-llama", device="cpu", seed=0, max_batch=8, block_size=16, num_blocks=128,
                     max_prefill_tokens=256, use_graphs=False, **kw)


@pytest.mark.parametrize("pipeline", [False, True])
def test_engine_json_mode_outputs_always_parse(pipeline):
    """Random-init weights (so no natural JSON): every json_mode answer is one JSON object, closed
    within its budget (2..40 tokens), mixed in a batch with unconstrained requests."""
    from django_assistant_bot_amd.engine.llm_engine import SamplingParams

    eng = _engine(pipeline_decode=pipeline)
    rids, js = [], []
    for i, budget in enumerate([2, 3, 5, 8, 13, 21, 40, 30]):
        sp = SamplingParams(max_new_tokens=budget, ignore_eos=True, json_mode=i != 5, seed=i)
        rids.append(eng.add_request(list(range(5, 30 + 7 * i)), sp))
        js.append(i != 5)
    while eng.has_unfinished():
        eng.step()
    for rid, j in zip(rids, js):
        out = eng.pop_output(rid)
        if not j:
            assert out.finish_reason == "length"
            continue
        obj = json.loads(out.text)
        assert isinstance(obj, dict), out.text
        assert out.finish_reason == "stop"
    assert eng.stats.get("json_broken", 0) == 0
    assert eng.blocks.num_free_blocks() == eng.blocks.num_blocks()


def test_provider_json_mode_single_attempt():
    """The app-layer provider (reference TransformersProvider contract) returns a parsed dict in one
    attempt with json_format=True."""
    import asyncio

    from assistant.ai.providers.transformers import TransformersProvider

    p = TransformersProvider("tiny-llama", device="cpu", seed=1, max_batch=4, max_model_len=512, use_graphs=False)
    res = asyncio.run(p.get_response([{"role": "user", "content": "Reply in JSON"}], max_tokens=24, json_format=True))
    assert isinstance(res.result, dict)
    assert res.usage["completion_tokens"] <= 24


def test_hf_byte_level_vocab_bytes(tmp_path):
    """Token byte strings of a byte-level BPE tokenizer.json (GPT-2 byte <-> unicode table)."""
    tokenizers = pytest.importorskip("tokenizers")
    from tokenizers import decoders, models, pre_tokenizers

    from django_assistant_bot_amd.engine.json_constraint import hf_token_bytes

    vocab = {"{": 0, "}": 1, "Ġ\"": 2, "Ã©": 3, "ĊĠ": 4, "<eos>": 5}
    tok = tokenizers.Tokenizer(models.BPE(vocab=vocab, merges=[]))
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tok.add_special_tokens(["<eos>"])
    got = hf_token_bytes(tok, 6)
    assert got == [b"{", b"}", b' "', "é".encode(), b"\n ", b""]


def test_wire_carries_json_mode():
    from django_assistant_bot_amd.engine.llm_engine import SamplingParams
    from django_assistant_bot_amd.parallel import wire

    it = wire.add_item(0, 7, [1, 2, 3], SamplingParams(json_mode=True, max_new_tokens=9))
    [(h, p)] = wire.unpack(*wire.pack([it]))
    _, rid, prompt, sp = wire.read_add(h, p)
    assert rid == 7 and prompt == [1, 2, 3] and sp.json_mode and sp.max_new_tokens == 9
    [(h, p)] = wire.unpack(*wire.pack([wire.add_item(0, 8, [4], SamplingParams())]))
    assert not wire.read_add(h, p)[3].json_mode
