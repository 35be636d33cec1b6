#!/usr/bin/env python
"""BASELINE config 1: all-MiniLM-L6 embeddings + brute-force cosine over 1k synthetic documents on
the CPU, through the service plumbing only (no GPU, no LLM).

The whole HTTP path runs in-process through FastAPI's test client: request validation, the
batching ``EmbedWorker`` and the JSON encoding of vectors.

* Ingest: ``POST /embeddings/`` for the documents in batches, then ``POST /index/docs/upsert``.
* Each query: ``POST /embeddings/`` for the question, then ``POST /index/docs/search`` (exact
  cosine top-k over the 1k rows).

Reported: sequential queries/s, p50, and throughput with ``--concurrency`` client threads.

    python benchmarks/plumbing_bench.py --docs 1000 --queries 200
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1000)
    ap.add_argument("--queries", type=int, default=200)
    ap.add_argument("--concurrency", type=int, default=8)
    ap.add_argument("--model", default="all-minilm-l6")
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--reference-rerun", action="store_true",
                    help="also time the reference algorithm: HF BertModel one text per forward (fp32, unmasked "
                         "mean pool, ai/embedders/transformers.py:15-25) + numpy cosine over the same 1k docs")
    args = ap.parse_args()

    os.environ["GPU_SERVICE_DEVICE"] = "cpu"
    os.environ["GPU_SERVICE_EMBEDDERS"] = args.model
    os.environ["GPU_SERVICE_PROVIDERS"] = ""
    import torch
    from fastapi.testclient import TestClient

    from bench import synth_text
    from gpu_service.main import app

    torch.set_num_threads(max(1, (os.cpu_count() or 4) // 2))
    rng = np.random.default_rng(0)
    docs = [synth_text(rng, int(rng.integers(80, 160))) for _ in range(args.docs)]
    questions = [synth_text(rng, int(rng.integers(6, 14))) + "?" for _ in range(args.queries)]
    with TestClient(app) as client:
        t0 = time.perf_counter()
        vecs = []
        for s in range(0, len(docs), 64):
            r = client.post("/embeddings/", json={"model": args.model, "texts": docs[s:s + 64]})
            r.raise_for_status()
            vecs += r.json()["embeddings"]
        r = client.post("/index/docs/upsert", json={"ids": list(range(len(docs))), "vectors": vecs})
        r.raise_for_status()
        ingest_s = time.perf_counter() - t0

        def one(q):
            t = time.perf_counter()
            e = client.post("/embeddings/", json={"model": args.model, "texts": [q]})
            e.raise_for_status()
            h = client.post("/index/docs/search", json={"queries": e.json()["embeddings"], "k": args.k})
            h.raise_for_status()
            assert len(h.json()["ids"][0]) == args.k
            return time.perf_counter() - t

        for q in questions[:10]:  # warm-up
            one(q)
        t0 = time.perf_counter()
        lat = [one(q) for q in questions]
        seq_s = time.perf_counter() - t0
        t0 = time.perf_counter()
        with ThreadPoolExecutor(args.concurrency) as ex:
            list(ex.map(one, questions))
        conc_s = time.perf_counter() - t0
        # the same work in-process (no HTTP): engine embed + index search
        from django_assistant_bot_amd.engine.serving import get_embed_worker
        from gpu_service.main import indexes

        eng, idx = get_embed_worker(args.model).engine, indexes["docs"]
        lat_ip = []
        for q in questions:
            t = time.perf_counter()
            idx.search(eng.embed([q]), args.k)
            lat_ip.append(time.perf_counter() - t)
    ref = {}
    if args.reference_rerun:
        ref = reference_rerun(args, docs, questions)
    print(json.dumps({
        "metric": "config 1: MiniLM-L6 embed + brute-force cosine over 1k docs, CPU, service plumbing",
        "value": round(args.queries / seq_s, 2), "unit": "queries/s (sequential)",
        "p50_latency_ms": round(1000 * float(np.median(lat)), 2),
        "p90_latency_ms": round(1000 * float(np.percentile(lat, 90)), 2),
        "concurrent_qps": round(args.queries / conc_s, 2), "concurrency": args.concurrency,
        "in_process": {"queries_per_s": round(len(lat_ip) / sum(lat_ip), 2),
                       "p50_latency_ms": round(1000 * float(np.median(lat_ip)), 2)},
        "ingest_docs_per_s": round(args.docs / ingest_s, 1),
        "config": {"model": args.model, "docs": args.docs, "k": args.k, "device": "cpu",
                   "data": "synthetic (random-init weights)"}, **ref}), flush=True)


def reference_rerun(args, docs, questions) -> dict:
    import torch
    import transformers

    from django_assistant_bot_amd.engine.tokenizer import Tokenizer
    from django_assistant_bot_amd.models.configs import encoder_config

    cfg = encoder_config(args.model)
    bert = transformers.BertModel(transformers.BertConfig(
        vocab_size=cfg.vocab_size, hidden_size=cfg.hidden, num_hidden_layers=cfg.layers, num_attention_heads=cfg.heads,
        intermediate_size=cfg.intermediate, max_position_embeddings=cfg.max_position)).eval()
    tok = Tokenizer.for_encoder(cfg)

    @torch.no_grad()
    def emb(text):
        ids = torch.tensor([tok.encode(text, max_len=cfg.max_position)])
        return bert(input_ids=ids).last_hidden_state.mean(dim=1).squeeze().numpy()

    t0 = time.perf_counter()
    mat = np.stack([emb(d) for d in docs])
    ingest_s = time.perf_counter() - t0
    mat /= np.linalg.norm(mat, axis=1, keepdims=True)
    lat = []
    t0 = time.perf_counter()
    for q in questions:
        t = time.perf_counter()
        e = emb(q)
        d = 1.0 - mat @ (e / np.linalg.norm(e))
        np.argsort(d)[: args.k]
        lat.append(time.perf_counter() - t)
    seq_s = time.perf_counter() - t0
    return {"reference_rerun": {"queries_per_s": round(len(questions) / seq_s, 2),
                                "p50_latency_ms": round(1000 * float(np.median(lat)), 2),
                                "ingest_docs_per_s": round(len(docs) / ingest_s, 1),
                                "note": "HF per-text embedding + numpy cosine, in-process (no HTTP, no DB)"}}


if __name__ == "__main__":
    main()
