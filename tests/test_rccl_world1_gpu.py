"""The RCCL data plane on the box's one MI355X: with ``DAB_FORCE_GROUP=1`` a
world-1 "nccl" process group forms, so every device-tensor collective branch that the 8-GPU node
runs executes here too instead of being skipped:

  * ``ShardedIndex.search`` (all_gather of the query block + the remainder rows, ``all_to_all_single``
    of packed partials, the merge) and ``search_replicated`` (all_reduce of the wide flag, ``gather``
    to the serving rank) -- exact against one unsharded ``VectorIndex``;
  * ``dist.barrier(device_ids=...)``, ``max_over_ranks`` / ``gather_floats`` / ``broadcast_int``;
  * the gpu_service node control plane (control broadcasts, the encoder ``gather``, index ingest and
    search through the sharded index) over HTTP;
  * ``bench.py --gpus 1`` reporting ``"backend": "nccl"``.

Reference: the only scaling knob of the reference is gunicorn workers
(/root/reference/gpu_service/gunicorn_conf.py:9); its retrieval is one pgvector scan
(/root/reference/assistant/rag/services/search_service.py:185-196)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, port, out_path):
    import traceback

    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      DAB_FORCE_GROUP="1", GPU_SERVICE_DEVICE="cuda")
    try:
        res = _collectives()
        res.update(_node())
        torch.save(res, out_path)
    except BaseException:
        with open(out_path + ".err", "w") as f:
            f.write(traceback.format_exc())
        raise


def _collectives():
    import torch.distributed as dist

    from django_assistant_bot_amd.engine.vector_index import VectorIndex
    from django_assistant_bot_amd.parallel import dist as pdist
    from django_assistant_bot_amd.parallel.sharded_index import ShardedIndex

    info = pdist.init(device_type="cuda")
    res = {"backend": info.backend, "pg_backend": dist.get_backend(), "world": dist.get_world_size()}
    pdist.barrier(info)
    res["max"] = pdist.max_over_ranks(3.5, info.device)
    res["gather"] = pdist.gather_floats(2.25, info.device)
    res["bcast"] = pdist.broadcast_int(7, None, info.device)
    g = torch.Generator().manual_seed(3)
    n, dim, k = 30000, 768, 50
    vecs = torch.randn(n, dim, generator=g)
    ids = np.arange(n) * 7 + 11
    docs = ids // 13
    groups = ((ids // 7) % 3).astype(np.int32)
    sh = ShardedIndex(dim, "cuda")
    sh.add(ids, vecs, doc_ids=docs, groups=groups)
    one = VectorIndex(dim, "cuda")
    one.add(ids, vecs, doc_ids=docs, groups=groups)
    res["comm_device"] = str(sh._comm_device())
    res["len"] = len(sh)
    q = torch.randn(20, dim, generator=g)  # 20 > SMALL_Q: the remainder all_gather runs too
    qg = (np.arange(20) % 3).astype(np.int32)
    a = sh.search(q, k, q_groups=qg)
    b = one.search(q, k, q_groups=qg)
    res["collectives"] = sh.stats.get("collectives", 0)
    res["search_ids_equal"] = bool(torch.equal(a[1].cpu(), b[1].cpu()))
    res["search_sims_err"] = float((a[0].float() - b[0].float()).abs().max())
    allowed = [ids[::5]] * 4
    c = sh.search_replicated(q[:4], k, allowed=allowed)
    d = one.search(q[:4], k, allowed=allowed)
    res["replicated_ids_equal"] = bool(torch.equal(c[1].cpu(), d[1].cpu()))
    res["merge_bytes"] = sh.stats["merge_bytes_recv"]
    return res


def _node():
    from fastapi import FastAPI
    from fastapi.testclient import TestClient

    from django_assistant_bot_amd.parallel.node import NodePlan
    from gpu_service import main as svc
    from gpu_service import node_main

    node = node_main.setup(embedders=["tiny-bert"], providers=[], plan=NodePlan(1), backend="nccl",
                           device_type="cuda", max_batch=8)
    res = {"node_grouped": node.grouped}
    try:
        app = FastAPI()
        for r in svc.app.routes:
            app.router.routes.append(r)
        c = TestClient(app)
        texts = [f"section {i} of the runbook, step {i % 7}" for i in range(64)]
        emb = c.post("/embeddings/", json={"model": "tiny-bert", "texts": texts}).json()["embeddings"]
        ref = node.embeds["tiny-bert"].embed(texts, out_dtype=torch.float32).cpu()
        res["node_embed_err"] = float((torch.tensor(emb) - ref).abs().max())
        ids = np.arange(len(texts)) * 3 + 1
        r = c.post("/index/kb/ingest", json={"model": "tiny-bert", "ids": ids.tolist(), "texts": texts,
                                             "doc_ids": (ids // 4).tolist()})
        res["node_count"] = r.json()["count"]
        s = c.post("/index/kb/search", json={"queries": ref[::5].tolist(), "k": 1}).json()
        res["node_top1"] = [x[0] for x in s["ids"]]
        res["node_want"] = ids[::5].tolist()
        res["node_commands"] = node.commands
    finally:
        node_main.teardown(node)
    return res


def test_world1_rccl_group_runs_every_collective_branch(tmp_path):
    out = str(tmp_path / "w1.pt")
    try:
        mp.spawn(_entry, args=(_free_port(), out), nprocs=1, join=True)
    except Exception:
        if os.path.exists(out + ".err"):
            print(open(out + ".err").read())
        raise
    res = torch.load(out, weights_only=True)
    print(res)
    assert res["backend"] == "nccl" and res["pg_backend"] == "nccl" and res["world"] == 1
    assert res["max"] == 3.5 and res["gather"] == [2.25] and res["bcast"] == 7
    assert res["comm_device"].startswith("cuda") and res["len"] == 30000
    assert res["collectives"] == 3  # query block + remainder all_gather, all_to_all of the partials
    assert res["search_ids_equal"] and res["search_sims_err"] < 1e-4  # (scores of a 20-query vs a gathered batch)
    assert res["replicated_ids_equal"] and res["merge_bytes"] > 0
    assert res["node_grouped"] and res["node_commands"] > 0
    assert res["node_embed_err"] < 1e-3
    assert res["node_count"] == 64 and res["node_top1"] == res["node_want"]


def test_bench_one_gpu_over_a_world1_rccl_group():
    cmd = [sys.executable, "bench.py", "--gpus", "1", "--embed-model", "tiny-bert", "--llm-model", "tiny-llama",
           "--index-rows", "20000", "--batch", "8", "--max-new-tokens", "8", "--steps", "1", "--warmup", "1"]
    p = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ, DAB_FORCE_GROUP="1"), capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    d = json.loads(lines[-1])
    assert d["backend"] == "nccl" and d["n_gpus"] == 1 and d["value"] > 0
    assert d["config"]["index"].startswith("sharded")
