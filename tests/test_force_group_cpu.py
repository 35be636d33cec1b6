"""``DAB_FORCE_GROUP=1`` on the CPU (gloo): a world-1 process group forms and ShardedIndex takes its
collective path (all_gather / all_to_all / gather) with results equal to the unsharded index; the
GPU twin with RCCL is tests/test_rccl_world1_gpu.py."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, port, out_path):
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      DAB_FORCE_GROUP="1")
    from django_assistant_bot_amd.engine.vector_index import VectorIndex
    from django_assistant_bot_amd.parallel import dist as pdist
    from django_assistant_bot_amd.parallel.sharded_index import ShardedIndex

    info = pdist.init(device_type="cpu")
    g = torch.Generator().manual_seed(1)
    n, dim, k = 3000, 64, 20
    vecs = torch.randn(n, dim, generator=g)
    ids = np.arange(n) * 3 + 5
    sh, one = ShardedIndex(dim, "cpu"), VectorIndex(dim, "cpu")
    sh.add(ids, vecs, doc_ids=ids // 7)
    one.add(ids, vecs, doc_ids=ids // 7)
    q = torch.randn(19, dim, generator=g)
    a, b = sh.search(q, k), one.search(q, k)
    c = sh.search_replicated(q[:3], k, doc_lt=[100, 200, 300])
    d = one.search(q[:3], k, doc_lt=[100, 200, 300])
    torch.save({"backend": info.backend, "collectives": sh.stats.get("collectives", 0),
                "eq": bool(torch.equal(a[1], b[1])), "eq_rep": bool(torch.equal(c[1], d[1])),
                "len": len(sh), "max": pdist.max_over_ranks(1.5, info.device)}, out_path)
    pdist.shutdown()


def test_world1_group_takes_the_collective_path(tmp_path):
    out = str(tmp_path / "w1.pt")
    mp.spawn(_entry, args=(_free_port(), out), nprocs=1, join=True)
    res = torch.load(out, weights_only=True)
    assert res["backend"] == "gloo" and res["collectives"] == 3
    assert res["eq"] and res["eq_rep"] and res["len"] == 3000 and res["max"] == 1.5


def test_no_group_without_the_opt_in(monkeypatch):
    from django_assistant_bot_amd.parallel import dist as pdist

    monkeypatch.delenv("DAB_FORCE_GROUP", raising=False)
    monkeypatch.setenv("WORLD_SIZE", "1")
    info = pdist.init(device_type="cpu")
    assert info.backend == "none" and not pdist.grouped()
