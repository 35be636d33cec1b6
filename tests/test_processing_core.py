"""Ingest pipeline without Django: wiki split -> format -> sentences -> questions -> embeddings ->
cross-document duplicate-question merge, on the in-memory repository with scripted LLM answers and the
hashed-bag-of-words fake embedder; plus the CSV parser and text helpers."""
import asyncio

import pytest

from assistant.ai.providers.fake import FakeAIProvider
from assistant.conf import configure, reset
from assistant.loading.csv_loader import normalize_title, read_rows
from assistant.processing.documents.processor import DefaultDocumentProcessor, get_document_processor
from assistant.processing.repository import MemoryIngestRepository, MemWiki
from assistant.processing.utils import estimated_min_length, language_ok, split_text_by_parts
from assistant.processing.wiki import ingest_wiki, split_wiki_document


@pytest.fixture(autouse=True)
def _fake():
    FakeAIProvider.reset()
    configure(DEFAULT_AI_MODEL="test", EMBEDDING_AI_MODEL="test", DOCUMENT_MAX_LENGTH=200)
    yield
    FakeAIProvider.reset()
    reset()


def test_text_helpers():
    parts = split_text_by_parts("a" * 300 + "\n" + "b" * 300 + "\nc\n", 500)
    assert parts == ["a" * 300 + "\n", "b" * 300 + "\nc\n"]
    assert all(len(p) <= 500 for p in split_text_by_parts("x\n" * 1000, 500))
    assert estimated_min_length("one two three") == min(15, int(13 * 0.8))
    assert language_ok(["Привет, как дела?"], "ru") and not language_ok(["Hello there my friend"], "ru")
    assert language_ok(["anything"], None)


def test_csv_rows(tmp_path):
    p = tmp_path / "kb.csv"
    p.write_text("﻿toc,name,content\n Shop  guide ,Delivery,  We ship daily.  \n\n"
                 "Shop guide,Returns,\"30 days, no questions\"\n", encoding="utf-8")
    assert list(read_rows(str(p))) == [("Shop guide", "Delivery", "We ship daily."),
                                       ("Shop guide", "Returns", "30 days, no questions")]
    bad = tmp_path / "bad.csv"
    bad.write_text("a,b\n1,2\n")
    with pytest.raises(ValueError):
        list(read_rows(str(bad)))
    assert normalize_title("  a \t b  ") == "a b"


def test_short_page_single_section():
    repo = MemoryIngestRepository()
    wiki = MemWiki(1, "Delivery", "We ship worldwide within five days.")
    proc = asyncio.run(split_wiki_document(wiki, repo))
    docs = [d for d in repo.documents.values() if d.processing is proc]
    assert [(d.name, d.content) for d in docs] == [("Delivery", wiki.content)]
    assert FakeAIProvider.requests == []  # no LLM call for a short page


def test_long_page_split_and_full_pipeline():
    repo = MemoryIngestRepository()
    body = ("Shipping takes five days to any country. Orders ship from our warehouse every day. " * 3
            + "\n" + "Returns are accepted within thirty days. Refunds go back to the original card. " * 3)
    wiki = MemWiki(7, "Store policy", body, path="Store / Store policy")
    section1 = "Shipping takes five days to any country. Orders ship from our warehouse every day."
    section2 = "Returns are accepted within thirty days. Refunds go back to the original card."
    FakeAIProvider.script([
        {"names": ["Shipping", "Returns"]},                 # split: section titles
        {"text": section1}, {"text": section2},              # split: section texts
        # section 1: format, sentences (1 part), questions (1 part)
        {"text": "**Shipping** takes five days to any country. Orders ship from our warehouse every day."},
        {"sentences": ["Store policy.", "Shipping takes five days to any country.",
                       "Orders ship from our warehouse every day.", "Shipping is daily."]},
        {"questions": ["How long does shipping take to another country?", "How often do orders ship?"]},
        # section 2
        {"text": section2},
        {"sentences": ["Store policy.", "Returns are accepted within thirty days.",
                       "Refunds go back to the original card.", "Returns policy."]},
        {"questions": ["How long does shipping take to another country?",   # exact duplicate of doc 1
                       "Within how many days are returns accepted?"]},
        2,  # placeholder never consumed if same text short-circuits the similarity check
    ])
    # merge: identical text -> no similarity call; then "which document is better?" -> 1 (keep the new one)
    FakeAIProvider._script.pop()
    FakeAIProvider.script([{"result": 1}])
    proc = asyncio.run(ingest_wiki(wiki, repo))
    assert proc.status == "completed"
    docs = sorted((d for d in repo.documents.values() if d.processing is proc), key=lambda d: d.id)
    assert [d.name for d in docs] == ["Shipping", "Returns"]
    assert docs[0].content.startswith("**Shipping**")  # the formatted text is kept (reference dropped it)
    sents = [r for r in repo.rows["sentences"].values()]
    assert len(sents) == 8 and all(r.embedding and len(r.embedding) == 768 for r in sents)
    assert [r.order for r in sents if r.document is docs[0]] == [0, 1, 2, 3]
    qs = {r.text: r for r in repo.rows["questions"].values()}
    # the duplicate kept in the second (newer) document, removed from the first
    dup = "How long does shipping take to another country?"
    assert dup in qs and qs[dup].document is docs[1]
    assert len(qs) == 3
    assert not FakeAIProvider._script  # every scripted answer consumed


def test_reprocessing_replaces_previous_run():
    repo = MemoryIngestRepository()
    wiki = MemWiki(3, "FAQ", "Short page about the store.")
    FakeAIProvider.script([{"text": "Short page about the store."},
                           {"sentences": ["FAQ.", "Short page about the store."]},
                           {"questions": ["What is this page about the store?"]}] * 2)
    first = asyncio.run(ingest_wiki(wiki, repo))
    second = asyncio.run(ingest_wiki(wiki, repo))
    assert first.id not in repo.processings and second.id in repo.processings
    assert all(d.processing is second for d in repo.documents.values())
    assert all(r.document.processing is second for k in repo.rows for r in repo.rows[k].values())


def test_processor_registry():
    get_document_processor.cache_clear()
    assert isinstance(get_document_processor("any"), DefaultDocumentProcessor)
    configure(DOCUMENT_PROCESSOR_CLASSES={"x": "assistant.processing.documents.processor.DefaultDocumentProcessor"})
    get_document_processor.cache_clear()
    assert isinstance(get_document_processor("x"), DefaultDocumentProcessor)
