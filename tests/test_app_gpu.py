"""The app layer end to end on the GPU engine: an ``AssistantBot`` console session whose fast and
strong models are ``engine:tiny-llama`` and whose knowledge base embeds with ``engine:tiny-bert`` into
an HBM index.  One RAG turn runs the reference's context pipeline: classify (constrained JSON, one
attempt), related-question search, choose-known-question (constrained JSON), broad document search,
FillInfo, final prompt, generation.  Random-init weights make the answer text meaningless, so the
checks are structural: every LLM call ran on the engine, the JSON steps parsed on their first try,
the final prompt carries the retrieved document, and the answer was posted.
Reference: /root/reference/assistant/bot/services/context_service/ (steps), assistant/bot/assistant_bot.py.
"""
import asyncio

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_rag_turn_on_the_engine(bpe_dir):
    from assistant.ai.providers import transformers as tp
    from assistant.bot.assistant_bot import AssistantBot
    from assistant.bot.platforms.api import CollectingPlatform
    from assistant.bot.session import BotSession
    from assistant.conf import configure, reset
    from assistant.rag.knowledge import KnowledgeDocument, MemoryKnowledgeBase, WikiRef
    from assistant.ai.services.ai_service import get_ai_embdedder, get_ai_provider

    from django_assistant_bot_amd.engine import serving
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine
    from django_assistant_bot_amd.models.configs import decoder_config
    from django_assistant_bot_amd.models.weights import random_decoder_weights

    # a byte-level BPE tokenizer (tests/conftest.py), so JSON Schemas are enforced token by token
    cfg = decoder_config("tiny-llama")
    eng = LLMEngine(cfg, device="cuda", seed=3, max_batch=8, max_model_len=2048, num_blocks=128, block_size=64,
                    weights=random_decoder_weights(cfg, "cuda", seed=3, interleave_mlp=True), checkpoint=bpe_dir)
    with serving._lock:
        serving._llm["tiny-llama@bpe"] = serving.LLMWorker(eng)
    configure(DEFAULT_AI_MODEL="engine:tiny-llama@bpe", EMBEDDING_AI_MODEL="engine:tiny-bert")
    calls = []
    orig = tp.TransformersProvider.get_response

    async def spy(self, messages, max_tokens=1024, json_format=False, **kw):
        res = await orig(self, messages, max_tokens=max_tokens, json_format=json_format, **kw)
        calls.append({"json": json_format, "schema": kw.get("json_schema") is not None,
                      "last": messages[-1]["content"], "result": res.result})
        return res

    tp.TransformersProvider.get_response = spy
    try:
        emb = get_ai_embdedder("engine:tiny-bert")
        dim = len(asyncio.run(emb.embeddings(["probe"]))[0])
        kb = MemoryKnowledgeBase(emb.embeddings, dim=dim, device="cuda")
        docs = [(KnowledgeDocument(1, "Shipping", "We ship worldwide in 5 days.", WikiRef("Store / Shipping", 10)),
                 ["how long does shipping take", "do you ship worldwide", "shipping time delivery days"]),
                (KnowledgeDocument(2, "Returns", "Returns are accepted within 30 days.", WikiRef("Store / Returns", 11)),
                 ["can i return an item", "return policy days", "refund for returns"])]
        for doc, qs in docs:
            asyncio.run(kb.add_document(doc, qs, "Store"))
        assert kb.index.vecs.is_cuda
        s = BotSession.in_memory(AssistantBot, CollectingPlatform(), system_text="You are a helpful bot.",
                                 language="en")
        s.dialog.instance.bot.knowledge = kb
        ans = asyncio.run(s.send("how long does shipping take"))
        assert ans is not None and isinstance(ans.text, str)
        assert len(s.platform.sent) == 1
        assert isinstance(get_ai_provider("engine:tiny-llama@bpe"), tp.TransformersProvider)
        assert eng.stats["decode_steps"] > 0 and eng.stats["graph_replays"] > 0
        json_calls = [c for c in calls if c["json"]]
        # classify (+ choose-known-question unless it was small talk): schema-constrained, so each
        # parses and meets the reference's repeat_until condition on its first attempt
        assert 1 <= len(json_calls) <= 2 and all(c["schema"] for c in json_calls), calls
        topic = json_calls[0]["result"]["topic"]
        assert topic in ("Small talk", "Store"), json_calls[0]
        assert not calls[-1]["json"]
        final = calls[-1]["last"]
        if topic == "Store":  # retrieval ran: the final prompt carries a retrieved document
            assert "We ship worldwide in 5 days." in final or "Returns are accepted within 30 days." in final, final
    finally:
        with serving._lock:
            serving._llm.pop("tiny-llama@bpe", None)
        tp.TransformersProvider.get_response = orig
        reset("DEFAULT_AI_MODEL", "EMBEDDING_AI_MODEL")
        torch.cuda.synchronize()
