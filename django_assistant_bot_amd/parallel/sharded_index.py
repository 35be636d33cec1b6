"""Vector index sharded across the GPUs of a node; partial top-k merged over RCCL / xGMI.

Row ownership: ``owner(id) = id % world``, so ingest on any rank routes each vector to the rank that
stores it and deletes need no broadcast.  Two search collectives:

* ``search`` -- every rank brings its own query batch (DP replicas of the RAG pipeline):
  all-gather the queries, scan the local shard for all of them, ``all_to_all`` each rank's partial
  top-k back to that rank only, merge W x k candidates with the top-k kernel.
* ``search_replicated`` -- every rank already holds the same batch (gpu_service's node group gets
  it with the control broadcast): scan, ``gather`` the partials to the serving rank, merge there.

Partials travel as (fp32 score bits, int32 id, int32 doc) = 12 B per hit (24 B only if an id
outgrows int32).  At k = 250 that is 3 KB per query per rank: the collectives are latency-bound
single calls over the fully connected xGMI links.  Reference counterpart: the per-query pgvector
scan + Python aggregation of /root/reference/assistant/rag/services/search_service.py:129-152,185-196.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from ..engine.vector_index import VectorIndex


class ShardedIndex:
    SMALL_Q = 16  # queries per rank that travel in the search's first (fixed-size) all_gather

    def __init__(self, dim: int, device=None, group=None, capacity: int = 4096, dtype=torch.bfloat16):
        self.group = group
        # the collective paths run on a group of > 1 ranks, or on any group under DAB_FORCE_GROUP;
        # a 1-rank (sub)group in a larger job searches locally (no gloo staging of a
        # world-1 collective)
        from .dist import force_group

        grouped = dist.is_available() and dist.is_initialized()
        self.distributed = grouped and (dist.get_world_size(group) > 1 or force_group())
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.world = dist.get_world_size(group) if self.distributed else 1
        self.local = VectorIndex(dim, device, capacity, dtype)
        self.device = self.local.device
        self.dim = dim
        self._max_key = 0  # largest id / doc id stored here: picks the 12 B or 24 B partial packing
        self.stats = {"merge_bytes_recv": 0}

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
        self._note_keys(ids[sel], d)
        self.local.add(ids[sel], v, d, g)
        return int(mine.sum())

    def _note_keys(self, ids, docs=None) -> None:
        if len(ids):
            self._max_key = max(self._max_key, int(np.max(ids)))
        if docs is not None and len(docs):
            self._max_key = max(self._max_key, int(np.max(docs)))

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
                docs_np = f.get_tensor("docs")[sel].numpy()
                idx._note_keys(ids_np[mine], docs_np)
                idx.local.add(ids_np[mine], f.get_tensor("vecs")[sel], docs_np, f.get_tensor("group")[sel].numpy())
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

    # ------------------------------------------------------------------ search
    def _pack(self, sims, ids, docs, k: int, wide: bool) -> torch.Tensor:
        """Partial top-k -> [q, k, 3] (score bits, id, doc): 12 B per hit as int32, 24 B only when an
        id does not fit in int32."""
        if sims.shape[1] < k:  # shard smaller than k: pad with empty hits
            pad = k - sims.shape[1]
            sims = torch.cat([sims, torch.full((sims.shape[0], pad), float("-inf"), device=sims.device)], 1)
            ids = torch.cat([ids, torch.full((ids.shape[0], pad), -1, dtype=ids.dtype, device=ids.device)], 1)
            docs = torch.cat([docs, torch.full((docs.shape[0], pad), -1, dtype=docs.dtype, device=docs.device)], 1)
        dt = torch.int64 if wide else torch.int32
        return torch.stack([sims.contiguous().view(torch.int32).to(dt), ids.to(dt), docs.to(dt)], -1)

    def _merge(self, cand: torch.Tensor, k: int):
        """cand [q, W*k, 3] packed partials of the same queries -> merged exact top-k."""
        cand = cand.to(self.device)
        cs = cand[..., 0].to(torch.int32).view(torch.float32).contiguous()
        kk = min(k, cs.shape[1], 1024)
        vals, pos = ops.topk_rows(cs, kk)
        pos = pos.long()
        out_ids = torch.gather(cand[..., 1], 1, pos).long()
        out_docs = torch.gather(cand[..., 2], 1, pos).long()
        dead = torch.isinf(vals)
        return vals, out_ids.masked_fill(dead, -1), out_docs.masked_fill(dead, -1)

    def _wide(self) -> bool:
        return self._max_key >= 2 ** 31

    @torch.inference_mode()
    def search(self, queries, k: int, q_groups=None):
        """Collective: every rank of the group calls it with its OWN (possibly empty) batch.

        1. all-gather the query batches (each rank scans its shard for every query of the node:
           per-GPU scan work is fixed as the node grows -- weak scaling);
        2. local exact top-k on the shard for all of them;
        3. ``all_to_all``: the partial top-k of rank r's queries goes to rank r only (W x less
           traffic than all-gathering every partial), packed in 12 B per hit;
        4. each rank merges the W partial lists of its own queries with the top-k kernel."""
        q = torch.as_tensor(queries).to(self.device, torch.float32)
        if q.ndim == 1:
            q = q[None]
        if not self.distributed:  # (a world-1 group, DAB_FORCE_GROUP, runs the collectives)
            return self.local.search(q, k, q_groups)
        cdev = self._comm_device()
        nq = q.shape[0]
        D = self.dim
        # 1. one all_gather of a fixed-size block: a header row (query count, wide-id flag) and up to
        #    SMALL_Q queries with their group in the last column.  Single-query searches (the app's
        #    per-message retrieval) thus cost two collectives (this + the all_to_all), not three;
        #    only a batch beyond SMALL_Q on some rank adds an all_gather of the remaining rows.
        S = self.SMALL_Q
        blk = torch.zeros((S + 1, D + 1), dtype=torch.float32, device=cdev)
        blk[0, 0] = float(nq)
        blk[0, 1] = float(self._wide())
        head = min(nq, S)
        grp = (torch.as_tensor(q_groups, dtype=torch.float32).to(cdev) if q_groups is not None
               else torch.full((nq,), -1.0, device=cdev))
        blk[1:1 + head, :D] = q[:head].to(cdev)
        blk[1:1 + head, D] = grp[:head]
        blks = [torch.empty_like(blk) for _ in range(self.world)]
        dist.all_gather(blks, blk, group=self.group)
        self.stats["collectives"] = 1
        hdr = torch.stack([b[0, :2] for b in blks]).cpu()  # the one host read of the call
        counts = [int(c) for c in hdr[:, 0].tolist()]
        wide = bool(hdr[:, 1].max().item())
        mx = max(counts)
        if mx == 0:
            z = torch.full((0, k), -1, dtype=torch.int64, device=self.device)
            return torch.full((0, k), float("-inf"), device=self.device), z, z.clone()
        parts = [b[1:1 + min(c, S)] for b, c in zip(blks, counts)]
        if mx > S:  # rows past SMALL_Q, padded to the largest remainder
            rest = torch.zeros((mx - S, D + 1), dtype=torch.float32, device=cdev)
            if nq > S:
                rest[:nq - S, :D] = q[S:].to(cdev)
                rest[:nq - S, D] = grp[S:]
            rests = [torch.empty_like(rest) for _ in range(self.world)]
            dist.all_gather(rests, rest, group=self.group)
            self.stats["collectives"] += 1
            parts = [torch.cat([p, r[:max(c - S, 0)]], 0) for p, r, c in zip(parts, rests, counts)]
        allq = torch.cat(parts, 0).to(self.device)  # real rows only, rank order
        # 2. local partial top-k for every query of the node
        sims, ids, docs = self.local.search(allq[:, :D], k, allq[:, D].to(torch.int32))
        packed = self._pack(sims, ids, docs, k, wide).to(cdev)  # [sum(counts), k, 3]
        # 3. route each rank's partials to that rank
        recv = torch.empty((self.world * nq, k, 3), dtype=packed.dtype, device=cdev)
        dist.all_to_all_single(recv, packed, output_split_sizes=[nq] * self.world, input_split_sizes=counts,
                               group=self.group)
        self.stats["collectives"] += 1
        self.stats["merge_bytes_recv"] = recv.numel() * recv.element_size()
        # 4. merge [nq, W*k] candidates
        cand = recv.view(self.world, nq, k, 3).permute(1, 0, 2, 3).reshape(nq, self.world * k, 3)
        return self._merge(cand, k)

    @torch.inference_mode()
    def search_replicated(self, queries, k: int, q_groups=None, allowed=None, doc_lt=None, dst: int = 0):
        """Collective for a batch every rank already holds (gpu_service: the request arrives with the
        control broadcast).  Each rank scans its shard with the full filter set (``allowed`` ids /
        ``doc_lt`` bounds are resolved against the local rows), the partials are gathered to ``dst``
        and merged there.  Returns the result on ``dst`` and None elsewhere."""
        q = torch.as_tensor(queries).to(self.device, torch.float32)
        if q.ndim == 1:
            q = q[None]
        if not self.distributed:  # (a world-1 group, DAB_FORCE_GROUP, runs the collectives)
            return self.local.search(q, k, q_groups, allowed=allowed, doc_lt=doc_lt)
        nq = q.shape[0]
        cdev = self._comm_device()
        flag = torch.tensor([int(self._wide())], dtype=torch.int64, device=cdev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
        wide = bool(flag.item())
        if len(self.local):
            sims, ids, docs = self.local.search(q, k, q_groups, allowed=allowed, doc_lt=doc_lt)
        else:
            sims = torch.full((nq, 0), float("-inf"), device=self.device)
            ids = docs = torch.full((nq, 0), -1, dtype=torch.int64, device=self.device)
        packed = self._pack(sims, ids, docs, k, wide).to(cdev)
        me = dist.get_rank(self.group) if self.group is not None else self.rank
        parts = [torch.empty_like(packed) for _ in range(self.world)] if me == dst else None
        gdst = dist.get_global_rank(self.group, dst) if self.group is not None else dst
        dist.gather(packed, parts, dst=gdst, group=self.group)
        if me != dst:
            return None
        self.stats["merge_bytes_recv"] = sum(p.numel() * p.element_size() for p in parts)
        cand = torch.stack(parts, 1).reshape(nq, self.world * k, 3)
        return self._merge(cand, k)
