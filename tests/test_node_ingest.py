"""Rank-local DP ingest (SURVEY.md 5.8 "DP ingest embedding", VERDICT r2 missing #3) on CPU gloo ranks.

``POST /index/{name}/ingest`` embeds texts and writes them into the sharded index.  Each text is
routed to the rank that owns its row (``id % S``); that rank embeds it and writes its own shard, so
with the default layout (every rank an encoder and a shard) no vector crosses a link.  With fewer
encoders than shards, only the rows of encoder-less shards travel, once, as vectors.
Reference: one embedder call per document then a bulk_update
(/root/reference/assistant/processing/documents/steps/embeddings.py:20-41,50-71).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytest.importorskip("fastapi")

W = 3
N = 240


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, embed_dp, out_path, device="cpu"):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), GPU_SERVICE_DEVICE=device)
    torch.set_num_threads(1)
    from django_assistant_bot_amd.parallel.node import NodePlan
    from gpu_service import node_main

    # device "cuda": every rank on the one GPU of the box (gloo control plane): the encoder runs
    # the native kernels and the shard is written from HBM
    node = node_main.setup(embedders=["tiny-bert"], providers=[], plan=NodePlan(world, embed_dp=embed_dp),
                           backend="gloo", device_type=device)
    try:
        if rank == 0:
            _drive(node, out_path)
        else:
            node.follow()
    finally:
        node_main.teardown(node)


def _drive(node, out_path):
    from fastapi import FastAPI
    from fastapi.testclient import TestClient

    from gpu_service import main as svc

    app = FastAPI()
    for r in svc.app.routes:
        app.router.routes.append(r)
    c = TestClient(app)
    res = {}
    ids = np.arange(N) * 7 + 2
    texts = [f"document {i} about topic {i % 13} and detail {i * 31 % 17}" for i in range(N)]
    half = N // 2
    r = c.post("/index/docs/ingest", json={"model": "tiny-bert", "ids": ids[:half].tolist(),
                                           "texts": texts[:half], "doc_ids": (ids[:half] // 10).tolist()})
    res["count1"] = r.json()["count"]
    r = c.post("/index/docs/ingest", json={"model": "tiny-bert", "ids": ids[half:].tolist(), "texts": texts[half:],
                                           "doc_ids": (ids[half:] // 10).tolist(), "return_vectors": True})
    body = r.json()
    res["count2"] = body["count"]
    got = torch.tensor(body["embeddings"])
    ref = node.embeds["tiny-bert"].embed(texts[half:], out_dtype=torch.float32).cpu()
    res["vec_err"] = float((got - ref).abs().max())
    # every row is found by its own embedding, with its doc id
    q = node.embeds["tiny-bert"].embed(texts[::10], out_dtype=torch.float32).cpu()
    s = c.post("/index/docs/search", json={"queries": q.tolist(), "k": 1}).json()
    res["top1"] = [x[0] for x in s["ids"]]
    res["top1_doc"] = [x[0] for x in s["doc_ids"]]
    res["want"] = ids[::10].tolist()
    # malformed payloads: 400, nothing broadcast
    cmds = node.commands
    bad = [{"model": "tiny-bert", "ids": [1, 2], "texts": ["a"]},
           {"model": "nope", "ids": [1], "texts": ["a"]},
           {"model": "tiny-bert", "ids": [-1], "texts": ["a"]},
           {"model": "tiny-bert", "ids": [1, 2], "texts": ["a", "b"], "groups": [0, -3]}]
    res["bad_status"] = [c.post("/index/docs/ingest", json=b).status_code for b in bad]
    res["bad_commands"] = node.commands - cmds
    st = node.command("stats")
    res["ingest_text_bytes"] = st[:, 4].tolist()
    res["ingest_vec_bytes"] = st[:, 5].tolist()
    res["owned"] = np.bincount(ids % W, minlength=W).tolist()
    res["dim"] = node.embeds["tiny-bert"].dim
    torch.save(res, out_path)


def _run(tmp_path, embed_dp, device="cpu"):
    out = str(tmp_path / "ingest.pt")
    mp.spawn(_entry, args=(W, _free_port(), embed_dp, out, device), nprocs=W, join=True)
    return torch.load(out, weights_only=True)


@pytest.mark.gpu
def test_rank_local_ingest_on_gpu(tmp_path):
    """Three ranks on the one GPU: native encoder, shards in HBM; the same checks as on CPU."""
    res = _run(tmp_path, 2, "cuda")
    assert res["count1"] == N // 2 and res["count2"] == N
    assert res["vec_err"] < 1e-3
    assert res["top1"] == res["want"]
    assert res["ingest_vec_bytes"][1] == 0 and res["ingest_vec_bytes"][2] == res["owned"][2] * res["dim"] * 4


@pytest.mark.parametrize("embed_dp", [0, 2])
def test_rank_local_ingest(tmp_path, embed_dp):
    res = _run(tmp_path, embed_dp)
    print({k: res[k] for k in ("ingest_text_bytes", "ingest_vec_bytes", "vec_err")})
    assert res["count1"] == N // 2 and res["count2"] == N
    assert res["vec_err"] < 1e-4
    assert res["top1"] == res["want"]
    assert res["top1_doc"] == [i // 10 for i in res["want"]]
    assert res["bad_status"] == [400] * 4 and res["bad_commands"] == 0
    D = W if embed_dp == 0 else embed_dp
    for r in range(1, W):
        if r < D:  # an encoder rank received the texts of its own rows, and no vectors
            assert res["ingest_text_bytes"][r] > 0
            assert res["ingest_vec_bytes"][r] == 0
        else:  # an encoder-less shard received exactly its rows' vectors, once
            assert res["ingest_text_bytes"][r] == 0
            assert res["ingest_vec_bytes"][r] == res["owned"][r] * res["dim"] * 4
