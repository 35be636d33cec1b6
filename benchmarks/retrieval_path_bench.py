"""Production retrieval path vs the raw index at 1M rows (BASELINE config 4's retrieval step).

Measures, per query (median over rounds, 1x MI355X):
  raw      VectorIndex.search(q, 250, q_groups=[g])                    (what bench.py's RAGPipeline does)
  service  assistant.storage.index.IndexService.search(qs, q, 250)     (the ORM bridge behind
           rag.services.search_service._objects_embedding_search), qs = the reference's hot filter
           (bot + COMPLETED) recognised from its where-tree -> one group compare, no pk list
  generic  IndexService.search with a filter the index cannot evaluate (pk allow-list of 1/2 the rows,
           fetched by one values_list and mapped to rows vectorised)
  kb       MemoryKnowledgeBase.search_documents (k = 5*5*10 = 250 questions + per-document aggregation)

The QuerySets are stubs carrying the same where-tree the Django ORM builds (Django is not installed
on the benchmark box); everything below the QuerySet is the production code.
"""
import asyncio
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from assistant.storage import index as index_mod  # noqa: E402
from assistant.rag.knowledge import KnowledgeDocument, MemoryKnowledgeBase  # noqa: E402
from tests.test_retrieval_filters import StubQS, _lookup  # noqa: E402


def med(fn, rounds=30):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    return float(np.median(ts))


def main(rows=1_000_000, dim=768, k=250):
    rng = np.random.default_rng(0)
    vecs = torch.randn(rows, dim, device="cuda")
    ids = np.arange(1, rows + 1, dtype=np.int64)
    docs = ids // 10
    bots = rng.integers(1, 3, rows)
    done = (rng.random(rows) < 0.9).astype(np.int64)
    groups = index_mod.row_group(bots, done)
    svc = index_mod.IndexService(backend="engine")
    svc._be.upsert("assistant_storage.question.embedding", ids, vecs, docs, groups)
    svc.ensure_loaded = lambda *a: None
    idx = svc._be._idx["assistant_storage.question.embedding"]
    q = torch.randn(dim).numpy()
    g = int(index_mod.row_group(1, 1))
    hot = StubQS([_lookup("assistant_storage.wikidocument", "bot", "exact", 1),
                  _lookup("assistant_storage.wikidocumentprocessing", "status", "exact", "completed")])
    gen = StubQS([_lookup("assistant_storage.question", "text", "icontains", "x")], pks=ids[::2].tolist())
    res = {"rows": rows, "k": k}
    res["raw_ms"] = med(lambda: idx.search(q[None], k, q_groups=[g]))
    res["service_ms"] = med(lambda: svc.search(hot, q, k))
    res["generic_ms"] = med(lambda: svc.search(gen, q, k), rounds=10)
    # knowledge-base path: index holds the same rows; documents are looked up per aggregated hit
    kb = MemoryKnowledgeBase(None, dim, device="cuda")
    kb.index = idx
    kb.questions = {int(i): ("q", int(d)) for i, d in zip(ids[:1], docs[:1])}
    kb.documents = {int(d): KnowledgeDocument(int(d), f"doc {d}", "") for d in np.unique(docs)}

    class KBQ(dict):  # question texts are not needed for the timing; avoid a 1M-entry dict
        def __getitem__(self, i):
            return ("q", int(i) // 10)
    kb.questions = KBQ()
    loop = asyncio.new_event_loop()  # a server's one event loop
    res["kb_ms"] = med(lambda: loop.run_until_complete(kb.search_documents("q", q, 5, 5)))
    res["service_over_raw"] = round(res["service_ms"] / res["raw_ms"], 3)
    res["kb_over_raw"] = round(res["kb_ms"] / res["raw_ms"], 3)
    res["threshold_searches"] = idx.stats["threshold_searches"]
    print(json.dumps({k2: (round(v, 3) if isinstance(v, float) else v) for k2, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
