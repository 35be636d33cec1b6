"""Data-parallel corpus embedding (document ingest / index build) across the GPUs of a node.

Rank r encodes the texts whose ids satisfy ``id % world == r`` -- exactly the rows ``ShardedIndex``
assigns to that rank -- so embeddings land in the owner's HBM index with no data movement at all;
only the row counts are all-reduced.  Within a rank, texts go through the engine's packed
variable-length batches (length-sorted, token budget), i.e. the MFMA encoder runs at large M.
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist


def owned_ids(n: int, rank: int, world: int, first_id: int = 0) -> np.ndarray:
    return np.arange(first_id + rank, first_id + n, world, dtype=np.int64) if world > 1 else \
        np.arange(first_id, first_id + n, dtype=np.int64)


@torch.inference_mode()
def embed_corpus(engine, text_of: Callable[[int], str], n: int, rank: int = 0, world: int = 1, index=None,
                 doc_of: Optional[Callable[[np.ndarray], np.ndarray]] = None, chunk: int = 65536,
                 first_id: int = 0, gather: bool = False):
    """Embed ids [first_id, first_id + n) with ``world`` ranks.

    text_of(id) -> text.  With ``index`` (a ShardedIndex / VectorIndex of this rank) the vectors are
    inserted as they are produced (doc ids from ``doc_of(ids)``); with ``gather`` the full [n, H] matrix
    is all-gathered (tests / small corpora).  Returns (local ids, local vectors or None, total rows)."""
    ids = owned_ids(n, rank, world, first_id)
    keep = [] if (index is None or gather) else None
    out_vecs = []
    # the next chunk is tokenised on a helper thread (the native tokenizer releases the GIL) while
    # this chunk's batches run on the GPU
    from concurrent.futures import ThreadPoolExecutor

    # the first block is small, so the GPU starts after ~1/8 of a block's tokenization instead of a
    # whole one (nothing overlaps the first block's tokenization)
    first = min(chunk, max(4096, chunk // 8))
    starts = [0] + list(range(first, len(ids), chunk)) if len(ids) > first else [0]
    bounds = starts[1:] + [len(ids)]

    def tokenize(k):
        return engine.tokenize([text_of(int(i)) for i in ids[starts[k]:bounds[k]]])

    pool = ThreadPoolExecutor(1) if len(starts) > 1 else None
    nxt = pool.submit(tokenize, 0) if pool else None
    for k, s in enumerate(starts):
        part = ids[s:bounds[k]]
        flat, offs = nxt.result() if pool else tokenize(k)
        if pool and k + 1 < len(starts):
            nxt = pool.submit(tokenize, k + 1)
        v = engine.embed_tokens(np.asarray(flat), np.asarray(offs), out_dtype=torch.float32)
        if index is not None:
            target = getattr(index, "local", index)  # ShardedIndex -> its local VectorIndex (we own these ids)
            docs = None if doc_of is None else doc_of(part)
            if hasattr(index, "_note_keys"):
                index._note_keys(part, docs)
            target.add(part, v, doc_ids=docs)
        if keep is not None or gather:
            out_vecs.append(v)
    if pool:
        pool.shutdown()
    local = torch.cat(out_vecs) if out_vecs else None
    total = len(ids)
    # the collectives run on the default group only when it IS this split's world of > 1 ranks (or a
    # world-1 group under DAB_FORCE_GROUP): a caller passing world=1 inside a larger job (its own
    # split) neither all-reduces with ranks that are not calling nor mis-sizes the gather
    from .dist import force_group

    if dist.is_initialized() and dist.get_world_size() == world and (world > 1 or force_group()):
        dev = engine.device if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor([total], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        total = int(t.item())
        if gather:
            H = engine.dim
            counts = [len(owned_ids(n, r, world, first_id)) for r in range(world)]
            buf = torch.zeros((max(counts), H), dtype=torch.float32, device=dev)
            if local is not None:
                buf[: len(ids)] = local.to(dev)
            parts = [torch.empty_like(buf) for _ in range(world)]
            dist.all_gather(parts, buf)
            full = torch.empty((n, H), dtype=torch.float32)
            for r in range(world):
                full[owned_ids(n, r, world, 0)] = parts[r][: counts[r]].cpu()
            return ids, full, total
    return ids, local, total
