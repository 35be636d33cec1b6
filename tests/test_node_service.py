"""gpu_service node mode (one process group over the node's GPUs) on CPU gloo ranks: the FastAPI app
on rank 0 drives the sharded index (upsert on one request, search on another), DP embeddings and
replicated / tensor-parallel generators; results must equal a single-process index / engine.
Reference: /root/reference/gpu_service/main.py:57-107 (endpoints), gunicorn_conf.py:9 (replicas)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytest.importorskip("fastapi")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _full(model):
    from django_assistant_bot_amd.models.configs import decoder_config
    from django_assistant_bot_amd.models.weights import random_decoder_weights

    cfg = decoder_config(model)
    return cfg, random_decoder_weights(cfg, dtype=torch.float32, seed=21)


def _shard(model, tp_rank, tp_size):
    """Every replica / TP group holds shards of ONE full model, so outputs can be compared with a
    single-process engine on the full weights."""
    from django_assistant_bot_amd.models.weights import shard_decoder_weights

    cfg, full = _full(model)
    return shard_decoder_weights(full, cfg, tp_rank, tp_size, interleave_mlp=True)


def _entry(rank, world, port, plan_kw, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), GPU_SERVICE_DEVICE="cpu")
    torch.set_num_threads(1)
    from django_assistant_bot_amd.parallel.node import NodePlan
    from gpu_service import node_main

    model = plan_kw.pop("model", "tiny-llama")
    node = node_main.setup(embedders=["tiny-bert"], providers=[model], plan=NodePlan(world, **plan_kw),
                           backend="gloo", device_type="cpu", llm_weights=_shard)
    try:
        if rank == 0:
            _drive(node, model, out_path)
        else:
            assert node.follow() > 0
    finally:
        node_main.teardown(node)


def _drive(node, model, out_path):
    from fastapi import FastAPI
    from fastapi.testclient import TestClient

    from django_assistant_bot_amd.engine import serving
    from django_assistant_bot_amd.engine.embedding_engine import EmbeddingEngine
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine, SamplingParams
    from django_assistant_bot_amd.engine.vector_index import VectorIndex
    from gpu_service import main as svc

    app = FastAPI()
    for r in svc.app.routes:
        app.router.routes.append(r)
    c = TestClient(app)
    res = {}
    # ---- index: two upserts (the second overwrites some ids), then searches on other requests
    g = torch.Generator().manual_seed(4)
    dim = 16
    ids = np.arange(1, 401) * 5
    vecs = torch.randn(400, dim, generator=g)
    docs = ids // 20
    groups = (ids // 5) % 2
    r1 = c.post("/index/q/upsert", json={"ids": ids[:250].tolist(), "vectors": vecs[:250].tolist(),
                                         "doc_ids": docs[:250].tolist(), "groups": groups[:250].tolist()})
    r2 = c.post("/index/q/upsert", json={"ids": ids[200:].tolist(), "vectors": vecs[200:].tolist(),
                                         "doc_ids": docs[200:].tolist(), "groups": groups[200:].tolist()})
    res["counts"] = (r1.json()["count"], r2.json()["count"])
    single = VectorIndex(dim, "cpu")
    single.add(ids, vecs, doc_ids=docs, groups=groups)
    q = torch.randn(5, dim, generator=g)
    body = {"queries": q.tolist(), "k": 30, "groups": [0, 1, 0, 1, 0],
            "allowed": [ids[::3].tolist()] * 5, "doc_lt": [int(docs[300])] * 5}
    got = c.post("/index/q/search", json=body).json()
    es, eids, edocs = single.search(q, 30, q_groups=body["groups"], allowed=body["allowed"], doc_lt=body["doc_lt"])
    exp_ids = [[x for x in row if x >= 0] for row in eids.tolist()]
    res["search_equal"] = got["ids"] == exp_ids
    res["search_docs_equal"] = got["doc_ids"] == [[x for x in row if x >= 0] for row in edocs.tolist()]
    res["dist_err"] = max(abs((1 - s) - d) for srow, drow in zip(es.tolist(), got["distances"])
                          for s, d in zip(srow, drow))
    res["removed"] = c.post("/index/q/delete", json={"ids": ids[:10].tolist()}).json()["removed"]
    single.remove(ids[:10])
    got = c.post("/index/q/search", json={"queries": q.tolist(), "k": 8}).json()
    res["after_delete_equal"] = got["ids"] == single.search(q, 8)[1].tolist()
    res["unknown_index"] = c.post("/index/zzz/search", json={"queries": q[:1].tolist(), "k": 3}).json()["ids"]
    # ---- embeddings: a large batch is split over the EMBED_DP ranks
    texts = [f"text number {i} about subject {i % 11} " * (1 + i % 5) for i in range(150)]
    got = np.asarray(c.post("/embeddings/", json={"model": "tiny-bert", "texts": texts}).json()["embeddings"])
    ref = EmbeddingEngine("tiny-bert", "cpu", seed=0).embed(texts).numpy()
    res["embed_err"] = float(np.abs(got - ref).max())
    res["embed_commands"] = node.commands
    # ---- dialog: one HTTP request, then concurrent requests spread over the replicas
    r = c.post("/dialog/", json={"model": model, "messages": [{"role": "user", "content": "hello there"}],
                                 "max_tokens": 5})
    res["dialog_tokens"] = r.json()["response"]["usage"]["completion_tokens"]
    worker = serving._llm[model]
    sp = SamplingParams(max_new_tokens=6, ignore_eos=True, do_sample=False, temperature=0.0)
    prompts = [list(range(3, 3 + n)) for n in (20, 7, 33, 12, 9)]
    futs = [worker.submit(p, sp) for p in prompts]
    outs = [f.result(timeout=120) for f in futs]
    eng = LLMEngine(model, "cpu", seed=0, max_batch=4, max_model_len=2048, use_graphs=False,
                    block_size=node.llms[model].block_size, weights=_shard(model, 0, 1))
    want = []
    for rid, p in zip([o.request_id for o in outs], prompts):
        eng.add_request(p, sp, request_id=rid)
    while eng.has_unfinished():
        eng.step()
    want = [eng.pop_output(o.request_id).token_ids for o in outs]
    res["gen_equal"] = [o.token_ids for o in outs] == want
    res["placed"] = worker.engine.stats_node["placed"]
    h = c.get("/health").json()
    res["health_indexes"] = h["indexes"]
    res["metrics_ok"] = 'dab_index_rows{index="q"} 390.0' in c.get("/metrics").text
    torch.save(res, out_path)


@pytest.mark.parametrize("world,plan_kw", [
    (2, {}),                                         # 2 shards, DP-2 embed, 2 generator replicas
    (4, {"index_shards": 3, "embed_dp": 2}),         # index / embed on subsets of the node
    (4, {"gen_tp": 2}),                              # 2 replicas x TP-2 generators
    (8, {"gen_tp": 8, "model": "tiny-llama-70b-layout", "embed_dp": 4}),  # one KV head per rank
])
def test_node_service_matches_single_process(tmp_path, world, plan_kw):
    out = str(tmp_path / "node.pt")
    mp.spawn(_entry, args=(world, _free_port(), dict(plan_kw), out), nprocs=world, join=True)
    res = torch.load(out, weights_only=True)
    assert res["counts"] == (250, 400)
    assert res["search_equal"] and res["search_docs_equal"] and res["dist_err"] < 1e-4
    assert res["removed"] == 10 and res["after_delete_equal"]
    assert res["unknown_index"] == [[]]
    assert res["embed_err"] < 1e-4
    assert res["dialog_tokens"] <= 5
    assert res["gen_equal"]
    replicas = world // plan_kw.get("gen_tp", 1)
    assert len(res["placed"]) == replicas and (replicas == 1 or min(res["placed"]) > 0)
    assert res["health_indexes"] == {"q": 390} and res["metrics_ok"]


@pytest.mark.gpu
def test_node_service_on_gpu(monkeypatch):
    """Node mode on the box's GPU (world 1): the same facades serve index, embeddings and dialog from
    the native kernels; results equal the plain engines on the same device."""
    from fastapi import FastAPI
    from fastapi.testclient import TestClient

    from django_assistant_bot_amd.engine import serving
    from django_assistant_bot_amd.engine.embedding_engine import EmbeddingEngine
    from django_assistant_bot_amd.engine.vector_index import VectorIndex
    from django_assistant_bot_amd.parallel.node import NodePlan
    from gpu_service import main as svc
    from gpu_service import node_main

    for k, v in dict(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0").items():
        monkeypatch.setenv(k, v)
    monkeypatch.setattr(serving, "_llm", {})
    monkeypatch.setattr(serving, "_emb", {})
    monkeypatch.setattr(svc, "embedders", {})
    monkeypatch.setattr(svc, "providers", {})
    monkeypatch.setattr(svc, "index_backend", svc.index_backend)
    node = node_main.setup(embedders=["tiny-bert"], providers=["tiny-llama"], plan=NodePlan(1), device_type="cuda")
    try:
        app = FastAPI()
        for r in svc.app.routes:
            app.router.routes.append(r)
        c = TestClient(app)
        g = torch.Generator().manual_seed(2)
        ids = np.arange(3000)
        vecs = torch.randn(3000, 64, generator=g)
        assert c.post("/index/n/upsert", json={"ids": ids.tolist(), "vectors": vecs.tolist(),
                                               "doc_ids": (ids // 10).tolist()}).json()["count"] == 3000
        q = torch.randn(4, 64, generator=g)
        got = c.post("/index/n/search", json={"queries": q.tolist(), "k": 20}).json()
        single = VectorIndex(64, "cuda")
        single.add(ids, vecs, doc_ids=ids // 10)
        assert got["ids"] == single.search(q, 20)[1].tolist()
        texts = [f"sentence {i} " * (i % 9 + 1) for i in range(40)]
        emb = np.asarray(c.post("/embeddings/", json={"model": "tiny-bert", "texts": texts}).json()["embeddings"])
        ref = EmbeddingEngine("tiny-bert", "cuda", seed=0).embed(texts).float().cpu().numpy()
        assert np.abs(emb - ref).max() < 1e-3
        r = c.post("/dialog/", json={"model": "tiny-llama", "messages": [{"role": "user", "content": "hi"}],
                                     "max_tokens": 7}).json()["response"]
        assert 0 < r["usage"]["completion_tokens"] <= 7
        assert node.llms["tiny-llama"].stats["decode_steps"] > 0
    finally:
        node_main.teardown(node)
