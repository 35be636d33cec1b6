"""Node control plane at world 4 on CPU gloo ranks (VERDICT r2 "next" #6, ADVICE r2 node payloads).

* every generator replica steps on its own: the per-step control cost on a replica leader (polling
  its request link, shipping outputs) stays well under a millisecond (bound 0.5 ms);
* an index search is answered while the replicas are in the middle of a generation;
* an upsert sends each index shard only the rows it owns (bytes per shard ~ 1/W of the batch);
* malformed /index payloads are answered 400 on rank 0 and never reach the other ranks: the group
  stays healthy and keeps serving;
* a /dialog/ request with a JSON schema the constrained decoder cannot compile is answered 400
  before it is queued; an ADD a replica still refuses fails only that request.
Reference: /root/reference/gpu_service/gunicorn_conf.py:9, /root/reference/assistant/rag/services/search_service.py:185-196.
"""
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytest.importorskip("fastapi")

W = 4
ROW_BYTES = 16 * 4 + 3 * 8  # fp32 vector (dim 16) + id, doc, group as int64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), GPU_SERVICE_DEVICE="cpu")
    torch.set_num_threads(1)
    from django_assistant_bot_amd.parallel.node import NodePlan
    from gpu_service import node_main

    node = node_main.setup(embedders=[], providers=["tiny-llama"], plan=NodePlan(world), backend="gloo",
                           device_type="cpu")
    # slow every decode step down so a generation is long enough to search in the middle of it
    node.llms["tiny-llama"].fault_hook = lambda eng: time.sleep(0.01)
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

    from django_assistant_bot_amd.engine import serving
    from django_assistant_bot_amd.engine.llm_engine import SamplingParams
    from gpu_service import main as svc

    app = FastAPI()
    for r in svc.app.routes:
        app.router.routes.append(r)
    c = TestClient(app)
    res = {}
    g = torch.Generator().manual_seed(7)
    n = 4000
    ids = np.arange(n) * 3 + 1
    vecs = torch.randn(n, 16, generator=g)
    r = c.post("/index/q/upsert", json={"ids": ids.tolist(), "vectors": vecs.tolist(),
                                        "doc_ids": (ids // 10).tolist(), "groups": (ids % 2).tolist()})
    res["count"] = r.json()["count"]
    st = node.command("stats")  # [rank, (ctrl_s, llm_steps, upsert bytes, embed bytes)]
    owned = np.bincount(ids % W, minlength=W)
    res["upsert_bytes"] = st[:, 2].tolist()
    res["owned_bytes"] = (owned * ROW_BYTES).tolist()
    # ---- malformed payloads: 400 on rank 0, nothing broadcast
    cmds = node.commands
    bad = [("/index/q/upsert", {"ids": [1, 2], "vectors": [[0.0] * 16, [1.0] * 16], "groups": [0, -1]}),
           ("/index/q/upsert", {"ids": [1, 2], "vectors": [[0.0] * 16, [1.0] * 16], "doc_ids": [1]}),
           ("/index/q/upsert", {"ids": [1], "vectors": [[0.0] * 8]}),
           ("/index/q/search", {"queries": [[0.0] * 16] * 2, "k": 5, "allowed": [[1, 2]]}),
           ("/index/q/search", {"queries": [[0.0] * 16], "k": 0}),
           ("/index/q/search", {"queries": [[0.0] * 16], "k": 5, "groups": [0, 1]}),
           ("/index/q/search", {"queries": [[0.0] * 15], "k": 5})]
    res["bad_status"] = [c.post(u, json=b).status_code for u, b in bad]
    res["bad_commands"] = node.commands - cmds
    res["health_after_bad"] = c.get("/health").status_code
    # ---- a search in the middle of a generation on every replica
    worker = serving._llm["tiny-llama"]
    sp = SamplingParams(max_new_tokens=40, ignore_eos=True, do_sample=False, temperature=0.0)
    futs = [worker.submit(list(range(3, 20 + i)), sp) for i in range(8)]
    time.sleep(0.3)
    t0 = time.perf_counter()
    q = torch.randn(3, 16, generator=g)
    got = c.post("/index/q/search", json={"queries": q.tolist(), "k": 10}).json()
    res["search_s"] = time.perf_counter() - t0
    res["search_rows"] = [len(x) for x in got["ids"]]
    res["gen_running_at_search"] = sum(not f.done() for f in futs)
    outs = [f.result(timeout=120) for f in futs]
    res["gen_tokens"] = [len(o.token_ids) for o in outs]
    # constrained requests travel the wire too (json_mode flag / schema text in the ADD item)
    import json

    jf = [worker.submit(list(range(3, 25)), SamplingParams(max_new_tokens=12, ignore_eos=True, json_mode=True)),
          worker.submit(list(range(4, 25)), SamplingParams(max_new_tokens=12, ignore_eos=True, json_schema={
              "type": "object", "properties": {"q": {"type": "integer"}}}))]
    res["json_ok"] = [isinstance(json.loads(f.result(timeout=120).text), dict) for f in jf]
    # ---- unsupported JSON schemas: 400 for the caller, the group keeps serving
    msg = [{"role": "user", "content": "hi"}]
    bad_schemas = [{"$ref": "#"}, {"type": "object", "properties": {"a": {}}}, {"type": "string"}, {"type": "array"}]
    res["schema_status"] = [c.post("/dialog/", json={"model": "tiny-llama", "messages": msg, "max_tokens": 8,
                                                     "json_schema": sch}).status_code for sch in bad_schemas]
    res["health_after_schema"] = c.get("/health").status_code
    # a refused ADD that slipped past the pre-check fails only its request, on whichever replica got it
    eng0 = worker.engine.engine
    orig = eng0.check_params
    eng0.check_params = lambda params, matcher=False: orig(params, matcher) if matcher else None
    try:
        rf = [worker.submit(list(range(3, 12)), SamplingParams(max_new_tokens=4, json_schema={"$ref": "#"}))
              for _ in range(W)]
        errs = []
        for f in rf:
            try:
                f.result(timeout=120)
                errs.append("")
            except Exception as exc:
                errs.append(str(exc))
        res["refused"] = ["refused" in e for e in errs]
    finally:
        eng0.check_params = orig
    after = worker.submit(list(range(3, 12)), SamplingParams(max_new_tokens=5, ignore_eos=True))
    res["gen_after_refused"] = len(after.result(timeout=120).token_ids)
    res["health_after_refused"] = c.get("/health").status_code
    res["placed"] = worker.engine.stats_node["placed"]
    st = node.command("stats")
    res["ctrl_s"] = st[:, 0].tolist()
    res["llm_steps"] = st[:, 1].tolist()
    torch.save(res, out_path)


def test_node_control_plane_world4(tmp_path):
    out = str(tmp_path / "ctrl.pt")
    mp.spawn(_entry, args=(W, _free_port(), out), nprocs=W, join=True)
    res = torch.load(out, weights_only=True)
    print({k: res[k] for k in ("upsert_bytes", "search_s", "gen_running_at_search", "ctrl_s", "llm_steps", "placed")})
    assert res["count"] == 4000
    # upsert: every shard received exactly its own rows (the old broadcast sent all 4000 to each)
    for r in range(1, W):
        assert res["upsert_bytes"][r] == res["owned_bytes"][r]
        assert res["upsert_bytes"][r] <= 1.05 * 4000 * ROW_BYTES / W
    assert res["bad_status"] == [400] * 7 and res["bad_commands"] == 0 and res["health_after_bad"] == 200
    # search answered while generations were still running on the replicas
    assert res["gen_running_at_search"] > 0 and res["search_rows"] == [10, 10, 10]
    assert res["search_s"] < 0.25, res["search_s"]
    assert res["gen_tokens"] == [40] * 8
    assert res["json_ok"] == [True, True]
    assert min(res["placed"]) > 0
    assert res["schema_status"] == [400] * 4 and res["health_after_schema"] == 200
    assert res["refused"] == [True] * W and res["gen_after_refused"] == 5 and res["health_after_refused"] == 200
    # per-step control cost on the replica leaders (ranks 1..3, each stepping its own replica)
    for r in range(1, W):
        assert res["llm_steps"][r] >= 40
        per_step_ms = 1000 * res["ctrl_s"][r] / res["llm_steps"][r]
        # typically 0.06-0.16 ms on this CPU container; the bound leaves room for a loaded host and
        # is still < 7 % of a 7.6 ms Llama-3-8B decode step (x3 when pytest-xdist workers share the 8
        # CPUs with the 4 ranks: only the serial run prices the control plane)
        bound = 1.5 if os.environ.get("PYTEST_XDIST_WORKER") else 0.5
        assert per_step_ms < bound, (r, per_step_ms)
