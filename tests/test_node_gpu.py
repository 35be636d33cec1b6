"""gpu_service node mode on the GPU path: two (or four) ranks share the box's one MI355X (gloo control and data
plane; RCCL needs a device per rank), each with a tiny-llama generator replica (HIP-graph decode) and
a tiny-bert encoder replica, the index sharded over both.  Over HTTP (FastAPI TestClient on rank 0):
a DP-split /embeddings/ batch equals one encoder's vectors, /dialog/ answers from both replicas
(plain and JSON mode; a JSON Schema degrades to JSON mode with the hash tokenizer), /index/*/ingest + search find every row, and /health stays 200.
Reference endpoints: /root/reference/gpu_service/main.py.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
pytest.importorskip("fastapi")

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, out_path, gen_tp=1):
    import traceback

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), GPU_SERVICE_DEVICE="cuda")
    from django_assistant_bot_amd.parallel.node import NodePlan
    from gpu_service import node_main

    node = node_main.setup(embedders=["tiny-bert"], providers=["tiny-llama"], plan=NodePlan(world, gen_tp=gen_tp),
                           backend="gloo", device_type="cuda", max_batch=8)
    try:
        if rank == 0:
            _drive(node, out_path)
        else:
            node.follow()
    except BaseException:
        with open(out_path + f".err{rank}", "w") as f:
            f.write(traceback.format_exc())
        raise
    finally:
        node_main.teardown(node)


def _drive(node, out_path):
    from fastapi import FastAPI
    from fastapi.testclient import TestClient

    from django_assistant_bot_amd.engine import serving
    from gpu_service import main as svc

    app = FastAPI()
    for r in svc.app.routes:
        app.router.routes.append(r)
    c = TestClient(app)
    res = {}
    texts = [f"chunk {i} of the manual, section {i % 9}" for i in range(100)]
    emb = c.post("/embeddings/", json={"model": "tiny-bert", "texts": texts}).json()["embeddings"]
    ref = node.embeds["tiny-bert"].embed(texts, out_dtype=torch.float32).cpu()
    res["embed_err"] = float((torch.tensor(emb) - ref).abs().max())
    msgs = [{"role": "user", "content": "hello there"}]
    outs = []
    for i in range(4):
        r = c.post("/dialog/", json={"model": "tiny-llama", "messages": msgs + [{"role": "user", "content": str(i)}],
                                     "max_tokens": 12})
        outs.append(r.status_code)
    res["dialog_status"] = outs
    rj = c.post("/dialog/", json={"model": "tiny-llama", "messages": msgs, "max_tokens": 16, "json_format": True})
    res["json_status"] = rj.status_code
    rs = c.post("/dialog/", json={"model": "tiny-llama", "messages": msgs, "max_tokens": 16, "json_format": True,
                                  "json_schema": {"type": "object", "properties": {"n": {"type": "integer"}},
                                                  "required": ["n"]}})
    res["schema_status"] = rs.status_code
    res["schema_body"] = json.dumps(rs.json())
    ids = np.arange(len(texts)) * 5 + 3
    r = c.post("/index/docs/ingest", json={"model": "tiny-bert", "ids": ids.tolist(), "texts": texts,
                                           "doc_ids": (ids // 10).tolist()})
    res["count"] = r.json()["count"]
    s = c.post("/index/docs/search", json={"queries": ref[::7].tolist(), "k": 1}).json()
    res["top1"] = [x[0] for x in s["ids"]]
    res["want"] = ids[::7].tolist()
    res["health"] = c.get("/health").status_code
    # concurrent requests spread over both replicas
    from django_assistant_bot_amd.engine.llm_engine import SamplingParams

    worker = serving._llm["tiny-llama"]
    futs = [worker.submit(list(range(3, 20 + i)), SamplingParams(max_new_tokens=10, ignore_eos=True))
            for i in range(6)]
    res["gen_tokens"] = [len(f.result(timeout=120).token_ids) for f in futs]
    res["placed"] = list(worker.engine.stats_node["placed"])
    torch.save(res, out_path)


@pytest.mark.parametrize("world,gen_tp", [(2, 1), (4, 2)])
def test_node_service_on_gpu(tmp_path, world, gen_tp):
    """(4, 2): two TP-2 generator replicas (leader-driven lock step inside each, IPC all-reduce in the
    decode graphs), four encoder replicas and four index shards."""
    out = str(tmp_path / "node.pt")
    try:
        mp.spawn(_entry, args=(world, _free_port(), out, gen_tp), nprocs=world, join=True)
    except Exception:
        for r in range(world):
            if os.path.exists(out + f".err{r}"):
                print(f"rank {r}:\n" + open(out + f".err{r}").read())
        raise
    res = torch.load(out, weights_only=True)
    print(res)
    assert res["embed_err"] < 1e-3
    assert res["dialog_status"] == [200] * 4 and res["json_status"] == 200 and res["schema_status"] == 200
    body = json.loads(res["schema_body"])["response"]
    assert isinstance(body["result"], dict), body  # the hash tokenizer degrades a schema to JSON mode
    assert res["count"] == 100 and res["top1"] == res["want"]
    assert res["health"] == 200
    assert res["gen_tokens"] == [10] * 6 and min(res["placed"]) > 0  # both replicas answered
