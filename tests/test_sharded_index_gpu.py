"""Sharded HBM index on the GPU path (BASELINE config 3's merge): W ranks
share the box's one MI355X (gloo transport; RCCL needs one device per rank), each holding its shard
in bf16 in the fragment layout the native score kernels read.  The merged top-k of the all_to_all
search (uneven per-rank batches, group filters, a batch past the small-query block) and of the
replicated serving search (allow-lists, document bounds) equals one unsharded index holding every
row.  Reference: pgvector ORDER BY CosineDistance LIMIT n
(/root/reference/assistant/rag/services/search_service.py:185-196).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, out_path):
    import faulthandler
    import traceback

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from django_assistant_bot_amd.parallel import dist as pdist

    faulthandler.enable()
    pdist.init(backend="gloo", device_type="cuda")
    try:
        _body(rank, out_path)
    except BaseException:
        with open(out_path + f".err{rank}", "w") as f:
            f.write(traceback.format_exc())
        raise
    finally:
        pdist.shutdown()


def _body(rank, out_path):
    from django_assistant_bot_amd.engine.vector_index import VectorIndex
    from django_assistant_bot_amd.parallel.sharded_index import ShardedIndex

    g = torch.Generator().manual_seed(5)
    n, dim, k = 20000, 768, 50
    vecs = torch.randn(n, dim, generator=g)
    ids = np.arange(7, 7 + n) * 3
    docs = ids // 11
    groups = ((ids // 3) % 3).astype(np.int32)
    idx = ShardedIndex(dim, "cuda")
    idx.add(ids, vecs, doc_ids=docs, groups=groups)
    single = VectorIndex(dim, "cuda")
    single.add(ids, vecs, doc_ids=docs, groups=groups)
    res = {"native": bool(idx.local.dtype == torch.bfloat16)}
    nq = 0 if rank == 1 else 2 + rank
    q = torch.randn(nq, dim, generator=torch.Generator().manual_seed(70 + rank))
    qg = [r % 3 for r in range(nq)]
    sims, got_ids, got_docs = idx.search(q, k, q_groups=qg)
    if nq:
        es, eids, edocs = single.search(q, k, q_groups=qg)
        res["own_equal"] = bool(torch.equal(got_ids.cpu(), eids.cpu()) and torch.equal(got_docs.cpu(), edocs.cpu()))
        res["own_err"] = float((sims.float().cpu() - es.float().cpu()).nan_to_num(0.0).abs().max())
    nq2 = 40 if rank == 0 else 1
    q2 = torch.randn(nq2, dim, generator=torch.Generator().manual_seed(170 + rank))
    _, i2, d2 = idx.search(q2, k)
    _, ei2, ed2 = single.search(q2, k)
    res["big_equal"] = bool(torch.equal(i2.cpu(), ei2.cpu()) and torch.equal(d2.cpu(), ed2.cpu()))
    qs = torch.randn(3, dim, generator=torch.Generator().manual_seed(99))
    allowed = [ids[::2].tolist(), ids[:3000].tolist(), ids.tolist()]
    doc_lt = [10 ** 9, 10 ** 9, int(docs[n // 2])]
    out = idx.search_replicated(qs, k, q_groups=None, allowed=allowed, doc_lt=doc_lt)
    if rank == 0:
        es, eids, edocs = single.search(qs, k, allowed=allowed, doc_lt=doc_lt)
        res["rep_equal"] = bool(torch.equal(out[1].cpu(), eids.cpu()) and torch.equal(out[2].cpu(), edocs.cpu()))
    torch.save(res, out_path + f".{rank}")


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_index_on_gpu_matches_single_index(tmp_path, world):
    out = str(tmp_path / "sidx.pt")
    try:
        mp.spawn(_entry, args=(world, _free_port(), out), nprocs=world, join=True)
    except Exception:
        for r in range(world):
            if os.path.exists(out + f".err{r}"):
                print(f"rank {r}:\n" + open(out + f".err{r}").read())
        raise
    for r in range(world):
        res = torch.load(out + f".{r}", weights_only=True)
        assert res["native"]
        if "own_equal" in res:
            assert res["own_equal"] and res["own_err"] < 1e-3, res
        assert res["big_equal"]
        if r == 0:
            assert res["rep_equal"]


def _dp_entry(rank, world, port, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from django_assistant_bot_amd.engine.embedding_engine import EmbeddingEngine
    from django_assistant_bot_amd.parallel import dist as pdist
    from django_assistant_bot_amd.parallel.dp_embed import embed_corpus
    from django_assistant_bot_amd.parallel.sharded_index import ShardedIndex

    info = pdist.init(backend="gloo", device_type="cuda")
    try:
        eng = EmbeddingEngine("tiny-bert", "cuda", seed=2)
        texts = [f"document number {i} about topic {i % 7}" for i in range(301)]
        idx = ShardedIndex(eng.dim, "cuda")
        ids, full, total = embed_corpus(eng, lambda i: texts[i], len(texts), info.rank, info.world_size, index=idx,
                                        gather=True, chunk=64)
        res = {"total": total, "local": len(idx.local), "own": len(ids)}
        if info.rank == 0:
            ref = EmbeddingEngine("tiny-bert", "cuda", seed=2).embed(texts)
            res["err"] = float((full.float().cpu() - ref.float().cpu()).abs().max())
        torch.save(res, out_path + f".{rank}")
    finally:
        pdist.shutdown()


def test_dp_corpus_embedding_on_gpu(tmp_path):
    """BASELINE config 2's DP ingest on the GPU path: each rank embeds its share with the native
    encoder (several tokenised chunks, the helper-thread pipeline) straight into its HBM shard."""
    out = str(tmp_path / "dp.pt")
    mp.spawn(_dp_entry, args=(2, _free_port(), out), nprocs=2, join=True)
    r0, r1 = (torch.load(out + f".{r}", weights_only=True) for r in range(2))
    assert r0["total"] == r1["total"] == 301
    assert r0["local"] == r0["own"] and r1["local"] == r1["own"] and r0["own"] + r1["own"] == 301
    assert r0["err"] < 1e-3


def _snap_entry(rank, world, port, directory):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from django_assistant_bot_amd.parallel import dist as pdist
    from django_assistant_bot_amd.parallel.sharded_index import ShardedIndex

    pdist.init(backend="gloo", device_type="cuda")
    try:
        g = torch.Generator().manual_seed(3)
        n, dim = 5000, 256
        vecs = torch.randn(n, dim, generator=g)
        ids = np.arange(n, dtype=np.int64) * 7 + 1
        idx = ShardedIndex(dim, "cuda")
        idx.add(ids, vecs, doc_ids=ids // 10, groups=np.zeros(n, dtype=np.int32))
        idx.remove(ids[:5])
        idx.save(directory)
        torch.distributed.barrier()
        back = ShardedIndex.load(directory, "cuda")
        q = torch.randn(4, dim, generator=g)
        for x, y in zip(idx.search(q, 20), back.search(q, 20)):
            assert torch.equal(x.cpu(), y.cpu())
    finally:
        pdist.shutdown()


def test_sharded_index_snapshot_on_gpu(tmp_path):
    """Per-rank safetensors shards written from HBM (fragment layout -> row-major) and read back."""
    mp.spawn(_snap_entry, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
