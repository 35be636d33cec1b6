"""Vector index sharded across the GPUs of a node; partial top-k merged with all-gather over xGMI.

Row ownership: ``owner(id) = id % world``, so ingest on any rank routes each vector to the rank that
stores it and deletes need no broadcast.  A search batch of every rank is answered in three steps:

  1. all-gather the query embeddings of all ranks (each rank scans its shard for ALL queries, so the
     per-GPU scan work stays constant as the node grows -- weak scaling);
  2. local fused score GEMM + exact top-k on the shard (``VectorIndex.search``);
  3. all-gather the packed partial results ([queries, k] x {similarity, id, doc}) and merge each
     rank's own queries with the top-k kernel over the W*k candidates.

Messages are tiny (k = 250 -> ~6 KB per query per rank): the collectives are latency-bound, one
all-gather each, which RCCL issues over the fully connected xGMI links.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from ..engine.vector_index import VectorIndex


class ShardedIndex:
    def __init__(self, dim: int, device=None, group=None, capacity: int = 4096, dtype=torch.bfloat16):
        self.group = group
        self.distributed = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.world = dist.get_world_size(group) if self.distributed else 1
        self.local = VectorIndex(dim, device, capacity, dtype)
        self.device = self.local.device
        self.dim = dim

    def owner(self, ids: np.ndarray) -> np.ndarray:
        return np.asarray(ids, dtype=np.int64) % self.world

    def add(self, ids, vectors, doc_ids=None, groups=None) -> int:
        """Adds the rows this rank owns (callers may pass the full set on every rank)."""
        ids = np.asarray(ids, dtype=np.int64).reshape(-1)
        mine = self.owner(ids) == self.rank
        if not mine.any():
            return 0
        sel = np.nonzero(mine)[0]
        v = torch.as_tensor(vectors)[torch.from_numpy(sel)] if len(sel) != len(ids) else vectors
        d = None if doc_ids is None else np.asarray(doc_ids)[sel]
        g = None if groups is None else np.asarray(groups)[sel]
        self.local.add(ids[sel], v, d, g)
        return int(mine.sum())

    # ------------------------------------------------------------------ snapshots
    def save(self, directory: str) -> str:
        """Every rank writes its shard as ``shard-RRR-of-WWW.safetensors`` (the index is a cache of
        the DB vectors; the snapshot is only for a fast warm start)."""
        import os

        os.makedirs(directory, exist_ok=True)
        self.local.compact()
        path = os.path.join(directory, f"shard-{self.rank:03d}-of-{self.world:03d}.safetensors")
        self.local.save(path)
        return path

    @classmethod
    def load(cls, directory: str, device=None, group=None) -> "ShardedIndex":
        """Warm start from a snapshot written by any world size: each rank reads every shard file
        (memory-mapped by safetensors) and keeps the rows it owns under the CURRENT world size."""
        import glob
        import os

        from safetensors import safe_open

        files = sorted(glob.glob(os.path.join(directory, "shard-*-of-*.safetensors")))
        if not files:
            raise FileNotFoundError(f"no index shards in {directory}")
        with safe_open(files[0], framework="pt") as f:
            dim = f.get_slice("vecs").get_shape()[1]
        idx = cls(dim, device, group)
        for path in files:
            with safe_open(path, framework="pt") as f:
                ids = f.get_tensor("ids")
                live = ids >= 0
                if not bool(live.any()):
                    continue
                ids_np = ids[live].numpy()
                mine = idx.owner(ids_np) == idx.rank
                if not mine.any():
                    continue
                sel = torch.nonzero(live).view(-1)[torch.from_numpy(np.nonzero(mine)[0])]
                idx.local.add(ids_np[mine], f.get_tensor("vecs")[sel], f.get_tensor("docs")[sel].numpy(),
                              f.get_tensor("group")[sel].numpy())
        return idx

    def remove(self, ids) -> int:
        ids = np.asarray(ids, dtype=np.int64).reshape(-1)
        return self.local.remove(ids[self.owner(ids) == self.rank])

    def __len__(self):
        if not self.distributed:
            return len(self.local)
        t = torch.tensor([len(self.local)], dtype=torch.int64, device=self._comm_device())
        dist.all_reduce(t, group=self.group)
        return int(t.item())

    def _comm_device(self):
        return self.device if (self.distributed and dist.get_backend(self.group) == "nccl") else torch.device("cpu")

    @torch.inference_mode()
    def search(self, queries, k: int, q_groups=None):
        """Collective: every rank of the group must call it (with its own, possibly empty, batch)."""
        q = torch.as_tensor(queries).to(self.device, torch.float32)
        if q.ndim == 1:
            q = q[None]
        if not self.distributed or self.world == 1:
            return self.local.search(q, k, q_groups)
        cdev = self._comm_device()
        nq = q.shape[0]
        # 1. gather every rank's queries (padded to the largest batch)
        counts = [torch.zeros(1, dtype=torch.int64, device=cdev) for _ in range(self.world)]
        dist.all_gather(counts, torch.tensor([nq], dtype=torch.int64, device=cdev), group=self.group)
        counts = [int(c.item()) for c in counts]
        mx = max(counts)
        if mx == 0:
            z = torch.full((0, k), -1, dtype=torch.int64, device=self.device)
            return torch.full((0, k), float("-inf"), device=self.device), z, z.clone()
        qg = torch.full((mx,), -1, dtype=torch.int32)
        if q_groups is not None:
            qg[:nq] = torch.as_tensor(q_groups, dtype=torch.int32)
        qpad = torch.zeros((mx, self.dim + 1), dtype=torch.float32, device=cdev)
        qpad[:nq, : self.dim] = q.to(cdev)
        qpad[:, self.dim] = qg.to(cdev).float()
        allq = [torch.empty_like(qpad) for _ in range(self.world)]
        dist.all_gather(allq, qpad, group=self.group)
        allq = torch.cat(allq, 0).to(self.device)
        # 2. local exact top-k for every query of the node
        kk = k
        sims, ids, docs = self.local.search(allq[:, : self.dim], kk, allq[:, self.dim].to(torch.int32))
        if sims.shape[1] < k:  # shard smaller than k: pad
            pad = k - sims.shape[1]
            sims = torch.cat([sims, torch.full((sims.shape[0], pad), float("-inf"), device=self.device)], 1)
            ids = torch.cat([ids, torch.full((ids.shape[0], pad), -1, dtype=torch.int64, device=self.device)], 1)
            docs = torch.cat([docs, torch.full((docs.shape[0], pad), -1, dtype=torch.int64, device=self.device)], 1)
        packed = torch.stack([sims.view(torch.int32).to(torch.int64), ids, docs], -1).to(cdev)  # [W*mx, k, 3]
        # 3. gather partials, merge own queries
        parts = [torch.empty_like(packed) for _ in range(self.world)]
        dist.all_gather(parts, packed, group=self.group)
        mine = torch.stack([p[self.rank * mx: self.rank * mx + nq] for p in parts], 1).to(self.device)  # [nq, W, k, 3]
        cand = mine.reshape(nq, self.world * k, 3)
        cs = cand[..., 0].to(torch.int32).view(torch.float32).contiguous()
        kk = min(k, cs.shape[1], 1024)
        vals, pos = ops.topk_rows(cs, kk)
        pos = pos.long()
        out_ids = torch.gather(cand[..., 1], 1, pos)
        out_docs = torch.gather(cand[..., 2], 1, pos)
        return vals, out_ids, out_docs
