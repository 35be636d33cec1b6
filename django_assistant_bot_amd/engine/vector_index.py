"""Exact in-HBM cosine top-k index: the pgvector replacement.

The reference stores 768-d vectors in PostgreSQL (``VectorField`` + HNSW m=16/ef_construction=64,
storage/models.py:32-58) and searches with ``qs.annotate(distance=CosineDistance(field, q))
.order_by('distance')[:n]`` (rag/services/search_service.py:185-196) -- approximate, on the CPU, one
query at a time.  Here rows live L2-normalised in bf16 in HBM (1M x 768 = 1.5 GB, noise next to
288 GB), every query of a batch is scored against every live row by the MFMA GEMM kernel with the
filter applied in its epilogue (row tombstones, per-query group = bot, optional allow-bitmask for
arbitrary QuerySet filters), and the exact top-k is selected by the radix-select kernel.
Recall is 1.0 by construction.  Distance semantics match pgvector: ``1 - cos``.

The index is a cache of the ORM (source of truth); it supports upsert, delete (tombstone + lazy
compaction), growth, and safetensors snapshots for warm starts.

On the GPU (bf16, dim % 128 == 0) the rows are held ONCE, in the ``ops.shuffle_weights`` fragment
layout: every 16-row x 32-k block is one coalesced 1 KB load for the 1..128-query scans
(index_scan.hip / the streaming GEMM's candidate epilogue) and one LDS-DMA piece for the phased
GEMM at >= 128 queries and the generic-filter score GEMM.  (Round 2 kept a row-major copy beside
it: 2x the index HBM.)  Only the 1/64 row sample of the threshold search is gathered row-major, and
cached until the next update.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .. import ops


class VectorIndex:
    def __init__(self, dim: int, device=None, capacity: int = 4096, dtype=torch.bfloat16):
        self.dim = dim
        self.device = torch.device(device if device is not None else ("cuda" if torch.cuda.is_available() else "cpu"))
        self.dtype = dtype
        self._cap = 0
        self.n = 0  # rows in use (live + tombstoned)
        self.stats = {"threshold_searches": 0, "threshold_overflows": 0}
        self.vecs = self.row_ids = self.row_docs = self.row_group = None
        self._row_of: dict[int, int] = {}
        self._sorted = None  # lazily built (sorted ids, rows) for vectorised id -> row lookups
        # fragment layout (see the module docstring) for bf16 GPU indexes of a 128-multiple width
        self.frag = self.device.type == "cuda" and dtype == torch.bfloat16 and dim % 128 == 0
        self._version = 0  # bumped by every update: invalidates the cached threshold sample
        self._sample = None
        self._dead = 0
        self._grow(max(64, capacity))

    # ------------------------------------------------------------------ storage
    def _grow(self, cap: int):
        cap = (cap + 255) // 256 * 256  # whole 256-row tiles for the fragment-layout scans / GEMMs
        dev = self.device
        vecs = torch.zeros((cap, self.dim), dtype=self.dtype, device=dev)
        ids = torch.full((cap,), -1, dtype=torch.int64, device=dev)
        docs = torch.full((cap,), -1, dtype=torch.int64, device=dev)
        grp = torch.full((cap,), -1, dtype=torch.int32, device=dev)
        if self.n:
            if self.frag:  # the first ceil(n / 16) 16-row blocks are a contiguous prefix
                e = -(-self.n // 16) * 16 * self.dim
                vecs.view(-1)[:e] = self.vecs.view(-1)[:e]
            else:
                vecs[: self.n] = self.vecs[: self.n]
            ids[: self.n] = self.row_ids[: self.n]
            docs[: self.n] = self.row_docs[: self.n]
            grp[: self.n] = self.row_group[: self.n]
        self.vecs, self.row_ids, self.row_docs, self.row_group = vecs, ids, docs, grp
        self._cap = cap

    # exact threshold search (no score matrix) for large indexes on the GPU: see _threshold_search
    threshold_search = True
    threshold_min_rows = 1 << 19
    # 1/64 of the rows (4 x fewer sample bytes and sample scores than 1/16 for ~4 x more candidates:
    # 10M rows x 512 queries 10.79 -> 9.15 ms, 128 queries 4.70 -> 4.59; profiles/index_search.md)
    sample_stride = 64

    def _put(self, rows: torch.Tensor, v: torch.Tensor) -> None:
        if self.frag:
            ops.shuffle_rows_into(self.vecs, rows, v)
        else:
            self.vecs[rows] = v

    def rows_data(self, rows) -> torch.Tensor:
        """Row-major copy of the given rows (any layout)."""
        rows = torch.as_tensor(rows, dtype=torch.int64, device=self.device)
        if not self.frag:
            return self.vecs[rows]
        R, K = self.vecs.shape
        v5 = self.vecs.view(R // 16, K // 32, 4, 16, 8)
        return v5[rows // 16, :, :, rows % 16, :].reshape(rows.numel(), K)

    def __len__(self) -> int:
        return len(self._row_of)

    def __contains__(self, item_id: int) -> bool:
        return int(item_id) in self._row_of

    def add(self, ids, vectors, doc_ids=None, groups=None) -> None:
        """Upsert rows.  ids: int64 [n]; vectors [n, dim] (any float dtype / device); doc_ids int64 [n]
        (document each row belongs to); groups int32 [n] (e.g. bot id; must be >= 0)."""
        ids = np.asarray(ids, dtype=np.int64).reshape(-1)
        n = len(ids)
        if n == 0:
            return
        v = torch.as_tensor(vectors).to(self.device, torch.float32).reshape(n, self.dim)
        v = F.normalize(v, dim=-1).to(self.dtype)
        docs = np.full(n, -1, dtype=np.int64) if doc_ids is None else np.asarray(doc_ids, dtype=np.int64)
        grp = np.zeros(n, dtype=np.int32) if groups is None else np.asarray(groups, dtype=np.int32)
        if (grp < 0).any():
            raise ValueError("groups must be >= 0 (negative marks deleted rows)")
        idl = ids.tolist()
        self._sorted = None
        if len(set(idl)) == n and not (self._row_of.keys() & set(idl)):
            # bulk insert of new ids (ingest): C-speed bookkeeping, contiguous rows
            if self.n + n > self._cap:
                self._grow(max(self.n + n, 2 * self._cap))
            rows = np.arange(self.n, self.n + n, dtype=np.int64)
            self._row_of.update(zip(idl, range(self.n, self.n + n)))
            self.n += n
        else:
            rows = np.empty(n, dtype=np.int64)
            fresh = []
            for i, x in enumerate(idl):
                r = self._row_of.get(x)
                if r is None:
                    fresh.append(i)
                else:
                    rows[i] = r
            if fresh:
                need = self.n + len(fresh)
                if need > self._cap:
                    self._grow(max(need, 2 * self._cap))
                for j, i in enumerate(fresh):
                    rows[i] = self.n + j
                    self._row_of[idl[i]] = self.n + j
                self.n += len(fresh)
        pin = self.device.type == "cuda"

        def dev(a):
            x = torch.from_numpy(np.ascontiguousarray(a))
            return (x.pin_memory() if pin else x).to(self.device, non_blocking=True)
        r = dev(rows)
        self._put(r, v)
        self._version += 1
        self.row_ids[r] = dev(ids)
        self.row_docs[r] = dev(docs)
        self.row_group[r] = dev(grp)

    def remove(self, ids) -> int:
        rows = [self._row_of.pop(int(x)) for x in np.asarray(ids).reshape(-1).tolist() if int(x) in self._row_of]
        if rows:
            self._sorted = None
            r = torch.as_tensor(rows, dtype=torch.int64, device=self.device)
            self._version += 1
            self.row_group[r] = -1
            self.row_ids[r] = -1
            self._dead += len(rows)
            if self._dead > 1024 and self._dead > self.n // 4:
                self.compact()
        return len(rows)

    def compact(self) -> None:
        live = (self.row_group[: self.n] >= 0).nonzero().flatten()
        m = live.numel()
        self._put(torch.arange(m, device=self.device), self.rows_data(live))
        self._version += 1
        self.row_ids[:m] = self.row_ids[live]
        self.row_docs[:m] = self.row_docs[live]
        self.row_group[:m] = self.row_group[live]
        self.row_group[m: self.n] = -1
        self.n = m
        self._dead = 0
        ids = self.row_ids[:m].cpu().numpy()
        self._row_of = {int(x): i for i, x in enumerate(ids.tolist())}
        self._sorted = None

    # ------------------------------------------------------------------ search
    def rows_of(self, ids) -> np.ndarray:
        """Row index of each live item id (ids that are not in the index are dropped).  Vectorised
        through a sorted (id, row) table rebuilt lazily after upserts / deletes."""
        ids = np.asarray(ids, dtype=np.int64).reshape(-1)
        if self._sorted is None:
            keys = np.fromiter(self._row_of.keys(), dtype=np.int64, count=len(self._row_of))
            vals = np.fromiter(self._row_of.values(), dtype=np.int64, count=len(self._row_of))
            order = np.argsort(keys, kind="stable")
            self._sorted = (keys[order], vals[order])
        keys, vals = self._sorted
        if not len(keys) or not len(ids):
            return np.zeros(0, dtype=np.int64)
        pos = np.searchsorted(keys, ids)
        pos = np.minimum(pos, len(keys) - 1)
        hit = keys[pos] == ids
        return vals[pos[hit]]

    def _pack_rows(self, row_mask: torch.Tensor) -> torch.Tensor:
        """bool [q, words*32] row mask (device) -> int32 bitmask [q, words] for the score epilogue."""
        q, nb = row_mask.shape
        w = row_mask.view(q, nb // 32, 32).to(torch.int64) << torch.arange(32, device=row_mask.device)
        packed = w.sum(-1)
        packed = packed - (packed >= (1 << 31)).to(torch.int64) * (1 << 32)
        return packed.to(torch.int32).contiguous()

    def allow_mask(self, allowed) -> torch.Tensor:
        """Per-query allowed item ids (sets, lists or int arrays) -> int32 bitmask [q, ceil(n/32)] over
        rows, built on the device (no per-id Python loop)."""
        words = (self.n + 31) // 32
        m = torch.zeros((len(allowed), words * 32), dtype=torch.bool, device=self.device)
        for qi, ids in enumerate(allowed):
            ids = np.fromiter(ids, dtype=np.int64) if isinstance(ids, (set, frozenset)) else ids
            rows = self.rows_of(ids)
            if len(rows):
                m[qi, torch.from_numpy(rows).to(self.device)] = True
        return self._pack_rows(m)

    def doc_lt_mask(self, limits) -> torch.Tensor:
        """Rows whose document id is < limits[q] (the ingest dedup filter ``document__id__lt``),
        bitmask built from the row metadata on the device."""
        words = (self.n + 31) // 32
        lim = torch.as_tensor(np.asarray(limits, dtype=np.int64), device=self.device)[:, None]
        m = torch.zeros((len(limits), words * 32), dtype=torch.bool, device=self.device)
        m[:, : self.n] = self.row_docs[None, : self.n] < lim
        return self._pack_rows(m)

    @torch.inference_mode()
    def scores(self, queries: torch.Tensor, q_groups=None, allowed=None, doc_lt=None) -> torch.Tensor:
        """fp32 cosine similarities [q, n] (-inf for filtered / deleted rows).  Filters: ``q_groups``
        (per-query row group, e.g. bot + status bit), ``allowed`` (per-query item ids), ``doc_lt``
        (per-query document-id bound); masks are ANDed."""
        q = F.normalize(torch.as_tensor(queries).to(self.device, torch.float32), dim=-1).to(self.dtype)
        qg = None if q_groups is None else torch.as_tensor(q_groups, dtype=torch.int32).to(self.device)
        allow = None if allowed is None else self.allow_mask(allowed)
        if doc_lt is not None:
            dm = self.doc_lt_mask(doc_lt)
            allow = dm if allow is None else allow & dm
        n = max(self.n, 4)
        n = (n + 3) // 4 * 4
        if self.frag:
            return ops.gemm_bt(q, self.vecs, epilogue=ops.EPI_SCORES, out_f32=True, row_group=self.row_group[:n],
                               q_group=qg, allow=allow, shuffled=True, n=n)
        return ops.gemm_bt(q, self.vecs[:n], epilogue=ops.EPI_SCORES, out_f32=True, row_group=self.row_group[:n],
                           q_group=qg, allow=allow)

    @torch.inference_mode()
    def search(self, queries, k: int, q_groups=None, allowed=None, doc_lt=None):
        """-> (similarity [q, k] fp32 desc, item ids [q, k] int64 (-1 = none), doc ids [q, k] int64).
        Group-only filters keep the exact threshold path (no score matrix) on large indexes."""
        queries = torch.as_tensor(queries)
        if queries.ndim == 1:
            queries = queries[None]
        nq = queries.shape[0]
        if self.n == 0 or k <= 0 or nq == 0:
            z = torch.full((nq, max(k, 0)), -1, dtype=torch.int64, device=self.device)
            return torch.full((nq, max(k, 0)), float("-inf"), device=self.device), z, z.clone()
        got = None
        if (self.device.type == "cuda" and allowed is None and doc_lt is None and self.n >= self.threshold_min_rows
                and k <= 1024 and self.threshold_search):
            got = self._threshold_search(queries, k, q_groups)
        if got is not None:
            vals, rows = got
        else:
            s = self.scores(queries, q_groups, allowed, doc_lt)
            kk = min(k, s.shape[1], 1024)
            vals, rows = ops.topk_rows(s, kk)
        rows = rows.long()
        ids = self.row_ids[rows]
        docs = self.row_docs[rows]
        dead = torch.isinf(vals)
        ids = ids.masked_fill(dead, -1)
        docs = docs.masked_fill(dead, -1)
        return vals, ids, docs

    def _threshold_search(self, queries, k: int, q_groups=None):
        """Exact top-k without the [q, n] score matrix.  The k-th best score over a strided 1/64
        sample of the rows is a lower bound for the k-th best over all rows.  So the score GEMM
        appends only scores >= that bound (about 16k per query on unstructured data), and an exact
        top-k runs over those.  A chunk whose candidate list overflows is retried or scanned on its
        own (``_threshold_chunk``)."""
        q = F.normalize(torch.as_tensor(queries).to(self.device, torch.float32), dim=-1).to(self.dtype)
        qg = None if q_groups is None else torch.as_tensor(q_groups, dtype=torch.int32).to(self.device)
        n4 = (self.n + 3) // 4 * 4
        ns = (self.n // self.sample_stride) // 4 * 4
        if ns < k:  # the sample's k-th best is a valid bound only if the sample holds k rows
            return None
        kk = k
        samp = self._sample_rows(ns)
        samp_group = self.row_group[: ns * self.sample_stride: self.sample_stride].contiguous()
        s_scores = ops.gemm_bt(q, samp, epilogue=ops.EPI_SCORES, out_f32=True, row_group=samp_group, q_group=qg)
        tv, _ = ops.topk_rows(s_scores, kk)
        del s_scores
        thr = tv[:, kk - 1].contiguous()
        # about k * stride scores clear the sample's k-th best (its rank in the whole index); the
        # lists hold twice that plus a fixed margin (the count's spread is ~sqrt(k) * stride).  Above
        # a byte budget for the [q, cap] lists the queries go through in chunks (k = 1024
        # at 512 queries asked for ~1 GB of candidate memory per search).
        cap = 2 * k * self.sample_stride + 4096
        per_chunk = max(1, self.CAND_BYTES // (8 * cap))
        parts = [self._threshold_chunk(queries, q, thr, k, cap, n4, qg, i, min(i + per_chunk, q.shape[0]), q_groups)
                 for i in range(0, q.shape[0], per_chunk)]
        if len(parts) == 1:
            return parts[0]
        return torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts])

    def _threshold_chunk(self, queries, q, thr, k: int, cap: int, n4: int, qg, i: int, j: int, q_groups):
        """Queries i:j of a threshold search.  A list that overflows its capacity (clustered data:
        far more rows than k x stride clear the sample's bound) is retried for THIS chunk with the
        capacity it needed, and past the memory budget this chunk alone takes the full score path
        -- never the whole batch."""
        qgs = None if qg is None else qg[i:j]
        got, cmax = self._threshold_candidates(q[i:j], thr[i:j], k, cap, n4, qgs)
        if got is None:
            cap2 = -(-cmax // 1024) * 1024
            if (j - i) * cap2 * 8 <= 4 * self.CAND_BYTES:
                self.stats["threshold_retries"] = self.stats.get("threshold_retries", 0) + 1
                got, _ = self._threshold_candidates(q[i:j], thr[i:j], k, cap2, n4, qgs)
        if got is None:  # this chunk through [chunk, n] score sub-batches
            self.stats["threshold_chunk_full"] = self.stats.get("threshold_chunk_full", 0) + 1
            step = max(1, (1 << 30) // (4 * max(1, self.n)))
            vs, rs = [], []
            for a in range(i, j, step):
                b = min(j, a + step)
                sc = self.scores(queries[a:b], None if q_groups is None else q_groups[a:b])
                v, r = ops.topk_rows(sc, min(k, sc.shape[1], 1024))
                vs.append(v)
                rs.append(r)
            got = (torch.cat(vs), torch.cat(rs))
        return got

    CAND_BYTES = 256 << 20  # candidate-list memory of one threshold search

    def _threshold_candidates(self, q, thr, k: int, cap: int, n4: int, qg):
        if self.frag:
            cand_val, cand_idx, cnt = ops.score_candidates_shuffled(q, self.vecs, n4, thr, cap, self.row_group[:n4], qg)
        else:
            cand_val, cand_idx, cnt = ops.score_candidates(q, self.vecs[:n4], thr, cap, self.row_group[:n4], qg)
        cmax = int(cnt.max())
        if cmax > cap:
            self.stats["threshold_overflows"] += 1
            return None, cmax
        self.stats["threshold_searches"] += 1
        # only the filled prefix of the lists (the longest one, ~16k of the 36k-entry capacity at
        # k = 250 on unstructured data) is ranked; shorter lists are -inf past their count
        n_use = min(cap, max(k, -(-cmax // 64) * 64))
        vals, pos = ops.topk_rows(cand_val[:, :n_use], min(k, n_use))
        rows = torch.gather(cand_idx, 1, pos.long())
        return (vals, rows.masked_fill(torch.isinf(vals), 0)), cmax

    def _sample_rows(self, ns: int) -> torch.Tensor:
        """The strided 1/64 row sample (row-major), cached until the next update."""
        key = (ns, self._version)
        if self._sample is None or self._sample[0] != key:
            rows = torch.arange(0, ns * self.sample_stride, self.sample_stride, device=self.device)
            with torch.inference_mode(False):
                self._sample = (key, self.rows_data(rows).contiguous())
        return self._sample[1]

    # ------------------------------------------------------------------ persistence
    def save(self, path: str) -> None:
        from safetensors.torch import save_file

        n = self.n
        save_file({"vecs": self.rows_data(torch.arange(n, device=self.device)).contiguous().cpu(),
                   "ids": self.row_ids[:n].cpu(),
                   "docs": self.row_docs[:n].cpu(), "group": self.row_group[:n].cpu()}, path,
                  metadata={"dim": str(self.dim)})

    @classmethod
    def load(cls, path: str, device=None) -> "VectorIndex":
        from safetensors.torch import load_file

        st = load_file(path)
        idx = cls(st["vecs"].shape[1], device, capacity=max(64, st["vecs"].shape[0]), dtype=st["vecs"].dtype)
        n = st["vecs"].shape[0]
        idx._put(torch.arange(n, device=idx.device), st["vecs"].to(idx.device))
        idx.row_ids[:n] = st["ids"].to(idx.device)
        idx.row_docs[:n] = st["docs"].to(idx.device)
        idx.row_group[:n] = st["group"].to(idx.device)
        idx.n = n
        idx._row_of = {int(x): i for i, x in enumerate(st["ids"].tolist()) if x >= 0}
        idx._sorted = None
        idx._dead = n - len(idx._row_of)
        return idx
