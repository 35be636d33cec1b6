"""Multi-process (gloo, CPU) checks of the distributed paths: tensor-parallel Llama forward and
leader/follower serving == the unsharded model (world 2, and world 4 / 8 on the Llama-3-70B head
layout, where TP 8 leaves one KV head per rank), ShardedIndex search == a single index, DP corpus
embedding == a single-rank embedding.  The same code runs over RCCL on GPUs (backend chosen by
parallel.dist.init)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fn, *args, world=WORLD):
    port = _free_port()
    mp.spawn(_entry, args=(fn, port, world) + args, nprocs=world, join=True)


def _entry(rank, fn, port, world, *args):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from django_assistant_bot_amd.parallel import dist as pdist

    info = pdist.init(backend="gloo", device_type="cpu")
    try:
        fn(info, *args)
    finally:
        pdist.shutdown()


# (world, model): the 70B head layout (64 query / 8 KV heads) at TP 4 and TP 8 (one KV head per rank)
TP_CASES = [(2, "tiny-llama"), (4, "tiny-llama-70b-layout"), (8, "tiny-llama-70b-layout")]


def _tp_body(info, out_path, model_name):
    from django_assistant_bot_amd.models.configs import decoder_config
    from django_assistant_bot_amd.models.llama import AttnMeta, KVCache, LlamaModel
    from django_assistant_bot_amd.models.weights import random_decoder_weights, shard_decoder_weights
    from django_assistant_bot_amd.parallel import dist as pdist

    W = info.world_size
    cfg = decoder_config(model_name)
    full = random_decoder_weights(cfg, dtype=torch.float32, seed=11)
    group, tp_rank, _ = pdist.tp_groups(W)
    shard = shard_decoder_weights(full, cfg, tp_rank, W)
    model = LlamaModel(cfg, shard, "cpu", tp_group=group, tp_size=W)
    ids = torch.arange(5, 45, dtype=torch.int32)
    T = ids.numel()
    kv = KVCache(cfg.layers, 4, cfg.kv_heads // W, 64, cfg.head_dim, "cpu", dtype=torch.float32)
    meta = AttnMeta(decode=False, positions=torch.arange(T, dtype=torch.int32), slots=torch.arange(T),
                    block_tables=torch.arange(4, dtype=torch.int32)[None], ctx_lens=torch.tensor([T], dtype=torch.int32),
                    cu_q=torch.tensor([0, T], dtype=torch.int32), max_q=T)
    h = model.forward(ids, meta, kv)
    local = model.logits(h)
    lg = model.full_logits(local)  # vocab-parallel head: every rank holds V / W of the rows
    if info.rank == 0:
        ref_model = LlamaModel(cfg, full, "cpu")
        kv2 = KVCache(cfg.layers, 4, cfg.kv_heads, 64, cfg.head_dim, "cpu", dtype=torch.float32)
        ref = ref_model.forward(ids, meta, kv2)
        lg_err = (lg - ref_model.logits(ref)).abs().max().item()
        torch.save({"err": (h - ref).abs().max().item(), "logits_err": lg_err, "vp": model.vocab_parallel,
                    "head_rows": model.lm_head.shape[0], "local_cols": local.shape[1]}, out_path)


@pytest.mark.parametrize("world,model_name", TP_CASES)
def test_tensor_parallel_forward_matches_full_model(tmp_path, world, model_name):
    out = str(tmp_path / "tp.pt")
    _run(_tp_body, out, model_name, world=world)
    res = torch.load(out, weights_only=True)
    assert res["err"] < 1e-4 and res["logits_err"] < 1e-4
    from django_assistant_bot_amd.models.configs import decoder_config

    V = decoder_config(model_name).vocab_size
    assert res["vp"] and res["head_rows"] == V // world and res["local_cols"] == V // world


def _index_body(info, out_path):
    from django_assistant_bot_amd.engine.vector_index import VectorIndex
    from django_assistant_bot_amd.parallel.sharded_index import ShardedIndex

    g = torch.Generator().manual_seed(3)
    n, dim = 3000, 32
    vecs = torch.randn(n, dim, generator=g)
    ids = np.arange(100, 100 + n)
    docs = ids // 7
    idx = ShardedIndex(dim, "cpu")
    idx.add(ids, vecs, doc_ids=docs)
    assert len(idx) == n
    q = torch.randn(3 + info.rank, dim, generator=torch.Generator().manual_seed(50 + info.rank))
    sims, got_ids, got_docs = idx.search(q, 25)
    single = VectorIndex(dim, "cpu")
    single.add(ids, vecs, doc_ids=docs)
    es, eids, edocs = single.search(q, 25)
    res = {"ids_equal": bool(torch.equal(got_ids, eids)), "docs_equal": bool(torch.equal(got_docs, edocs)),
           "sims_err": float((sims - es).abs().max())}
    torch.save(res, out_path + f".{info.rank}")


def test_sharded_index_matches_single_index(tmp_path):
    out = str(tmp_path / "idx.pt")
    _run(_index_body, out)
    for r in range(WORLD):
        res = torch.load(out + f".{r}", weights_only=True)
        assert res["ids_equal"] and res["docs_equal"] and res["sims_err"] < 1e-5


def _index_merge_body(info, out_path):
    """all_to_all merge at world W: uneven per-rank batches (one rank empty), group filters, and
    the replicated (serving) search with allow-lists / doc bounds gathered to rank 0."""
    from django_assistant_bot_amd.engine.vector_index import VectorIndex
    from django_assistant_bot_amd.parallel.sharded_index import ShardedIndex

    W = info.world_size
    g = torch.Generator().manual_seed(5)
    n, dim, k = 2000, 32, 40
    vecs = torch.randn(n, dim, generator=g)
    ids = np.arange(7, 7 + n) * 3
    docs = ids // 11
    groups = ((ids // 3) % 3).astype(np.int32)
    idx = ShardedIndex(dim, "cpu")
    idx.add(ids, vecs, doc_ids=docs, groups=groups)
    single = VectorIndex(dim, "cpu")
    single.add(ids, vecs, doc_ids=docs, groups=groups)
    nq = 0 if info.rank == 1 else 2 + info.rank
    q = torch.randn(nq, dim, generator=torch.Generator().manual_seed(70 + info.rank))
    qg = [r % 3 for r in range(nq)]
    res = {}
    sims, got_ids, got_docs = idx.search(q, k, q_groups=qg)
    res["nq"] = nq
    if nq:
        es, eids, edocs = single.search(q, k, q_groups=qg)
        res["own_equal"] = bool(torch.equal(got_ids, eids) and torch.equal(got_docs, edocs))
        res["own_err"] = float((sims - es).nan_to_num(0.0).abs().max())
    res["bytes"] = idx.stats["merge_bytes_recv"]
    res["coll_small"] = idx.stats["collectives"]
    # a batch past SMALL_Q on one rank: the remaining rows travel in one extra all_gather
    nq2 = 40 if info.rank == 0 else 1
    q2 = torch.randn(nq2, dim, generator=torch.Generator().manual_seed(170 + info.rank))
    s2, i2, d2 = idx.search(q2, k)
    e2, ei2, ed2 = single.search(q2, k)
    res["big_equal"] = bool(torch.equal(i2, ei2) and torch.equal(d2, ed2))
    res["coll_big"] = idx.stats["collectives"]
    # single-query latency (the app's per-message retrieval)
    import time

    q1 = torch.randn(1, dim, generator=torch.Generator().manual_seed(7))
    idx.search(q1, k)
    torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(20):
        idx.search(q1, k)
    res["single_ms"] = (time.perf_counter() - t0) / 20 * 1e3
    # serving path: the same batch on every rank, filters resolved per shard
    qs = torch.randn(3, dim, generator=torch.Generator().manual_seed(99))
    allowed = [ids[::2].tolist(), ids[:300].tolist(), ids.tolist()]
    doc_lt = [10 ** 9, 10 ** 9, int(docs[n // 2])]
    out = idx.search_replicated(qs, k, q_groups=None, allowed=allowed, doc_lt=doc_lt)
    if info.rank == 0:
        es, eids, edocs = single.search(qs, k, allowed=allowed, doc_lt=doc_lt)
        res["rep_equal"] = bool(torch.equal(out[1], eids) and torch.equal(out[2], edocs))
        res["rep_err"] = float((out[0] - es).nan_to_num(0.0).abs().max())
    else:
        res["rep_none"] = out is None
    torch.save(res, out_path + f".{info.rank}")


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_index_all_to_all_merge(tmp_path, world):
    out = str(tmp_path / "merge.pt")
    _run(_index_merge_body, out, world=world)
    k = 40
    for r in range(world):
        res = torch.load(out + f".{r}", weights_only=True)
        if res["nq"]:
            assert res["own_equal"] and res["own_err"] < 1e-5
        # each rank receives only the partials of its own queries: W x nq x k x 12 B
        assert res["bytes"] == world * res["nq"] * k * 12
        assert res["coll_small"] == 2 and res["coll_big"] == 3 and res["big_equal"]
        if r == 0:
            print(f"W={world}: single-query sharded search {res['single_ms']:.2f} ms (gloo, CPU)")
        if r == 0:
            assert res["rep_equal"] and res["rep_err"] < 1e-5
        else:
            assert res["rep_none"]


def _dp_embed_body(info, out_path):
    from django_assistant_bot_amd.engine.embedding_engine import EmbeddingEngine
    from django_assistant_bot_amd.parallel.dp_embed import embed_corpus
    from django_assistant_bot_amd.parallel.sharded_index import ShardedIndex

    eng = EmbeddingEngine("tiny-bert", "cpu", seed=2)
    texts = [f"document number {i} about topic {i % 7}" for i in range(37)]
    idx = ShardedIndex(eng.dim, "cpu")
    ids, full, total = embed_corpus(eng, lambda i: texts[i], len(texts), info.rank, info.world_size, index=idx,
                                    gather=True)
    assert total == 37 and len(idx) == 37 and len(idx.local) == len(ids)
    if info.rank == 0:
        ref = EmbeddingEngine("tiny-bert", "cpu", seed=2).embed(texts)
        torch.save({"err": float((full - ref).abs().max())}, out_path)


def test_dp_corpus_embedding_matches_single_rank(tmp_path):
    out = str(tmp_path / "dp.pt")
    _run(_dp_embed_body, out)
    assert torch.load(out, weights_only=True)["err"] < 1e-5


def _snapshot_body(info, directory):
    from django_assistant_bot_amd.parallel.sharded_index import ShardedIndex

    g = torch.Generator().manual_seed(3)
    n, dim = 600, 32
    vecs = torch.randn(n, dim, generator=g)
    ids = np.arange(n, dtype=np.int64) * 7 + 1
    idx = ShardedIndex(dim, "cpu")
    idx.add(ids, vecs, doc_ids=ids // 10, groups=np.zeros(n, dtype=np.int32))
    idx.remove(ids[:5])
    idx.save(directory)
    torch.distributed.barrier()
    back = ShardedIndex.load(directory, "cpu")  # same world size
    q = torch.randn(4, dim, generator=g)
    a, b = idx.search(q, 20), back.search(q, 20)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_sharded_index_snapshot_reshards(tmp_path):
    d = str(tmp_path / "snap")
    _run(_snapshot_body, d)
    from django_assistant_bot_amd.engine.vector_index import VectorIndex
    from django_assistant_bot_amd.parallel.sharded_index import ShardedIndex

    single = ShardedIndex.load(d, "cpu")  # world 1: both shard files merged into one
    assert len(single) == 595
    g = torch.Generator().manual_seed(3)
    n, dim = 600, 32
    vecs = torch.randn(n, dim, generator=g)
    ids = np.arange(n, dtype=np.int64) * 7 + 1
    ref = VectorIndex(dim, "cpu")
    ref.add(ids[5:], vecs[5:], doc_ids=ids[5:] // 10, groups=np.zeros(n - 5, dtype=np.int32))
    q = torch.randn(4, dim, generator=g)
    s1, i1, d1 = single.search(q, 20)
    s2, i2, d2 = ref.search(q, 20)
    assert torch.equal(i1, i2) and torch.equal(d1, d2) and torch.allclose(s1, s2)


def _tp_engine(cfg, weights, **kw):
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine

    return LLMEngine(cfg, device="cpu", weights=weights, max_batch=4, block_size=16, num_blocks=64,
                     max_prefill_tokens=64, use_graphs=False, interleaved_mlp=False, **kw)


def _tp_requests():
    from django_assistant_bot_amd.engine.llm_engine import SamplingParams

    sp = SamplingParams(max_new_tokens=7, do_sample=False, temperature=0.0, ignore_eos=True)
    return [(list(range(5, 5 + n)), sp) for n in (30, 90, 12, 50, 3)]  # 90 > 64: chunked prefill


def _drive(engine):
    reqs = _tp_requests()
    rids = [engine.add_request(p, sp) for p, sp in reqs[:3]]
    for _ in range(2):
        engine.step()
    rids += [engine.add_request(p, sp) for p, sp in reqs[3:]]  # arrive while others decode
    engine.abort(rids[2])  # a client that went away
    while engine.has_unfinished():
        engine.step()
    return [engine.pop_output(r).token_ids for r in rids]


def _tp_serving_body(info, out_path, model_name):
    from django_assistant_bot_amd.models.configs import decoder_config
    from django_assistant_bot_amd.models.weights import random_decoder_weights, shard_decoder_weights
    from django_assistant_bot_amd.parallel import dist as pdist
    from django_assistant_bot_amd.parallel import tp_serving

    W = info.world_size
    cfg = decoder_config(model_name)
    full = random_decoder_weights(cfg, dtype=torch.float32, seed=21)
    group, tp_rank, _ = pdist.tp_groups(W)
    ctrl = tp_serving.control_group(list(range(W)))
    eng = _tp_engine(cfg, shard_decoder_weights(full, cfg, tp_rank, W), tp_group=group, tp_size=W,
                     tp_rank=tp_rank)
    if info.rank == 0:
        leader = tp_serving.TPLeader(eng, ctrl)
        toks = _drive(leader)
        leader.shutdown()
        torch.save(toks, out_path)
    else:
        steps = tp_serving.follow(eng, ctrl)
        assert steps > 5
        assert not eng.has_unfinished()


@pytest.mark.parametrize("world,model_name", TP_CASES)
def test_tp_leader_follower_serving_matches_single_process(tmp_path, world, model_name):
    out = str(tmp_path / "tp_tokens.pt")
    _run(_tp_serving_body, out, model_name, world=world)
    from django_assistant_bot_amd.models.configs import decoder_config
    from django_assistant_bot_amd.models.weights import random_decoder_weights

    cfg = decoder_config(model_name)
    ref = _drive(_tp_engine(cfg, random_decoder_weights(cfg, dtype=torch.float32, seed=21)))
    got = torch.load(out, weights_only=True)
    assert got == ref
    assert [len(t) for t in got] == [7, 7, len(got[2]), 7, 7] and len(got[2]) < 7
