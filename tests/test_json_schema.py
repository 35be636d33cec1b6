"""JSON-Schema-constrained decoding (engine/json_schema.py -> csrc/runtime/json_grammar.cpp
SchemaAutomaton): the compiled automaton against instances / non-instances of each schema, masks
against a brute force with the budget rule, and engine generations for the app's two fast-model
JSON steps (reference steps/classify.py:41-45, steps/choose_known_question.py:45-50: their
``repeat_until`` conditions hold after ONE generation)."""
import asyncio
import json
import random

import numpy as np
import pytest

from django_assistant_bot_amd.engine.json_schema import compile_schema
from django_assistant_bot_amd.ops import native

CLASSIFY = {"type": "object", "properties": {"topic": {"type": "string", "enum": ["Small talk", "Billing", "Доступ"]}},
            "required": ["topic"]}
KNOWN = {"type": "object", "properties": {"question": {"anyOf": [{"type": "integer", "minimum": 1, "maximum": 5},
                                                                 {"type": "null"}]}}, "required": ["question"]}
RICH = {"type": "object", "properties": {
    "name": {"type": "string", "maxLength": 6},
    "score": {"type": "number"},
    "n": {"type": "integer"},
    "ok": {"type": "boolean"},
    "tags": {"type": "array", "items": {"type": "string"}, "maxItems": 3},
    "sub": {"type": "object", "properties": {"x": {"type": ["integer", "null"]}}},
    "kind": {"const": "doc"}}}


def _auto(schema, toks=None):
    n = native()
    toks = toks if toks is not None else [bytes([b]) for b in range(256)] + [b""]
    v = n.JsonVocab(toks, [len(toks) - 1])
    return n.SchemaAutomaton(v, *compile_schema(schema))


@pytest.mark.parametrize("schema,good,bad", [
    (CLASSIFY, [{"topic": "Billing"}, {"topic": "Доступ"}, {"topic": "Small talk"}],
     [{"topic": "billing"}, {"topic": 3}, {"topc": "Billing"}, {}]),
    (KNOWN, [{"question": 1}, {"question": 5}, {"question": None}],
     [{"question": 0}, {"question": 6}, {"question": "1"}, {"question": 1.5}]),
    (RICH, [{"name": "ab\"c", "score": -1.5e3, "n": 0, "ok": True, "tags": [], "sub": {"x": None}, "kind": "doc"},
            {"name": "", "score": 2, "n": -17, "ok": False, "tags": ["a", "b", "c"], "sub": {"x": 4}, "kind": "doc"}],
     [{"name": "toolong", "score": 1, "n": 1, "ok": True, "tags": [], "sub": {"x": 1}, "kind": "doc"},
      {"name": "a", "score": 1, "n": 1.5, "ok": True, "tags": [], "sub": {"x": 1}, "kind": "doc"},
      {"name": "a", "score": 1, "n": 1, "ok": True, "tags": ["a", "b", "c", "d"], "sub": {"x": 1}, "kind": "doc"},
      {"name": "a", "score": 1, "n": 1, "ok": True, "tags": [], "sub": {"x": 1}, "kind": "dog"}]),
])
def test_automaton_instances(schema, good, bad):
    a = _auto(schema)
    for obj in good:
        for indent in (None, 1):
            text = json.dumps(obj, ensure_ascii=False, indent=indent).encode()
            assert a.accepts(text), text
    for obj in bad:
        assert not a.accepts(json.dumps(obj, ensure_ascii=False).encode()), obj
    assert not a.accepts(b"")


def test_unsupported_schemas_are_refused():
    for s in ({"type": "string"}, {"type": "object", "properties": {"a": {"$ref": "#"}}},
              {"type": "object", "properties": {"a": {}}}):
        with pytest.raises(ValueError):
            compile_schema(s)


def _mask_set(m, V, remaining):
    buf = np.zeros(-(-V // 32), dtype=np.int32)
    cnt = m.fill_mask(remaining, buf.ctypes.data)
    s = set(np.nonzero(np.unpackbits(buf.view(np.uint8), bitorder="little")[:V])[0].tolist())
    assert cnt == len(s)
    return s


def test_schema_masks_match_brute_force_and_close_in_budget():
    toks = [bytes([c]) for c in b'{}[]:," \nabcdefghijklmnopqrstuvwxyz0123456789-.'] + [
        b'{"', b'":', b'"}', b'"topic"', b' "', b'Bill', b'ing"', b'Small', b' talk', b'null', b'}\n',
        "Доступ".encode(), b"\\", b"question", b""]
    n = native()
    v = n.JsonVocab(toks, [len(toks) - 1])
    rng = random.Random(0)
    for schema in (CLASSIFY, KNOWN):
        a = n.SchemaAutomaton(v, *compile_schema(schema))
        for trial in range(25):
            m = n.SchemaMatcher(a)
            prefix = []
            # the budget rule counts one token per completion byte: enough budget to close at worst
            budget = m.completion_len() + rng.randrange(1, 10)
            for step in range(budget):
                remaining = budget - step
                got = _mask_set(m, len(toks), remaining)
                want = set()
                base = m.completion_len()
                for t in range(len(toks)):
                    if not toks[t]:
                        continue
                    mm = n.SchemaMatcher(a)
                    assert all(mm.advance(p) for p in prefix)
                    if mm.advance(t) and mm.completion_len() <= min(remaining - 1, base + 64):
                        want.add(t)
                assert got == want, (schema, prefix, remaining)
                t = rng.choice(sorted(got))
                assert m.advance(t)
                prefix.append(t)
                if m.done():
                    break
            assert m.done(), b"".join(toks[t] for t in prefix)
            obj = json.loads(m.text())
            assert obj == json.loads(b"".join(toks[t] for t in prefix))


@pytest.mark.parametrize("pipeline", [False, True])
def test_engine_schema_outputs_satisfy_the_reference_conditions(pipeline, bpe_dir):
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine, SamplingParams
    from django_assistant_bot_amd.models.configs import decoder_config
    from django_assistant_bot_amd.models.weights import random_decoder_weights

    cfg = decoder_config("tiny-llama")
    eng = LLMEngine(cfg, device="cpu", seed=0, max_batch=8, block_size=16, num_blocks=160,
                    weights=random_decoder_weights(cfg, "cpu", seed=0, interleave_mlp=True), checkpoint=bpe_dir,
                    max_prefill_tokens=256, use_graphs=False, pipeline_decode=pipeline)
    assert eng.tokenizer.byte_exact
    schemas = [CLASSIFY, KNOWN, RICH]
    rids = []
    for i in range(9):
        sp = SamplingParams(max_new_tokens=[24, 12, 120][i % 3], ignore_eos=True, seed=i, json_schema=schemas[i % 3])
        rids.append(eng.add_request(list(range(5, 30 + 9 * i)), sp))
    rids.append(eng.add_request(list(range(5, 40)), SamplingParams(max_new_tokens=7, ignore_eos=True)))
    while eng.has_unfinished():
        eng.step()
    for i, rid in enumerate(rids[:-1]):
        out = eng.pop_output(rid)
        obj = json.loads(out.text)
        if i % 3 == 0:
            assert obj["topic"] in CLASSIFY["properties"]["topic"]["enum"]
        elif i % 3 == 1:
            q = obj["question"]
            assert q is None or (isinstance(q, int) and 1 <= q <= 5)
        else:
            assert list(obj) == list(RICH["properties"]) and obj["kind"] == "doc" and len(obj["name"]) <= 6
        assert out.finish_reason == "stop"
    assert len(eng.pop_output(rids[-1]).token_ids) == 7
    assert eng.stats.get("json_broken", 0) == 0


def test_hash_tokenizer_degrades_schema_to_json_mode():
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine, SamplingParams

    eng = LLMEngine("tiny-llama", device="cpu", seed=0, max_batch=4, block_size=16, num_blocks=64,
                    max_prefill_tokens=256, use_graphs=False)
    rid = eng.add_request(list(range(5, 30)), SamplingParams(max_new_tokens=20, json_schema=KNOWN, ignore_eos=True))
    while eng.has_unfinished():
        eng.step()
    assert isinstance(json.loads(eng.pop_output(rid).text), dict)
    assert eng.stats.get("json_broken", 0) == 0


def test_provider_and_steps_pass_schemas(bpe_dir):
    from assistant.ai.providers.base import accepts_json_schema
    from assistant.ai.providers.fake import FakeAIProvider
    from assistant.ai.providers.transformers import TransformersProvider
    from django_assistant_bot_amd.engine import serving
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine
    from django_assistant_bot_amd.models.configs import decoder_config
    from django_assistant_bot_amd.models.weights import random_decoder_weights

    cfg = decoder_config("tiny-llama")
    eng = LLMEngine(cfg, device="cpu", seed=3, max_batch=4, max_model_len=512, use_graphs=False, num_blocks=64,
                    block_size=16, weights=random_decoder_weights(cfg, "cpu", seed=3, interleave_mlp=True),
                    checkpoint=bpe_dir)
    with serving._lock:
        serving._llm["tiny-llama@bpe"] = serving.LLMWorker(eng)
    p = TransformersProvider("tiny-llama@bpe")
    for _ in range(3):  # the reference's condition holds on the first attempt, every time
        res = asyncio.run(p.get_response([{"role": "user", "content": "?"}], max_tokens=16, json_schema=KNOWN))
        q = res.result["question"]
        assert q is None or (isinstance(q, int) and 1 <= q <= 5), res.result
    assert accepts_json_schema(p.get_response) and accepts_json_schema(FakeAIProvider().get_response)

    class Legacy:  # a custom provider with the reference's signature
        async def get_response(self, messages, max_tokens=1024, json_format=False):
            return None

    assert not accepts_json_schema(Legacy().get_response)


def test_wire_carries_json_schema():
    from django_assistant_bot_amd.engine.llm_engine import SamplingParams
    from django_assistant_bot_amd.parallel import wire

    [(h, p)] = wire.unpack(*wire.pack([wire.add_item(1, 9, [3, 4], SamplingParams(json_schema=CLASSIFY,
                                                                                   stop_token_ids=(7,)))]))
    _, rid, prompt, sp = wire.read_add(h, p)
    assert rid == 9 and prompt == [3, 4] and sp.stop_token_ids == (7,)
    assert json.loads(sp.json_schema) == CLASSIFY


def test_app_step_schemas_compile_and_match_their_conditions():
    """The schemas the app's fast-model steps send (ClassifyStep: the topic list as an enum;
    ChooseKnownQuestionStep: 1..n or null) accept exactly what the reference's conditions accept."""
    from assistant.bot.services.context_service.steps.choose_known_question import ChooseKnownQuestionStep
    from assistant.bot.services.context_service.steps.classify import ClassifyStep

    a = _auto(ClassifyStep.schema(["Small talk", "Оплата", 'Quote "x"']))
    assert a.accepts(json.dumps({"topic": 'Quote "x"'}).encode())
    assert a.accepts(json.dumps({"topic": "Оплата"}, ensure_ascii=False).encode())
    assert not a.accepts(b'{"topic": "Other"}')
    a = _auto(ChooseKnownQuestionStep.schema(3))
    for q in (1, 2, 3, None):
        obj = {"question": q}
        assert a.accepts(json.dumps(obj).encode()) and ChooseKnownQuestionStep._condition(
            type("R", (), {"result": obj})())
    assert not a.accepts(b'{"question": 4}') and not a.accepts(b'{"question": "1"}')
