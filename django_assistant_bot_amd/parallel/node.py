"""One engine process group over the GPUs of a node: gpu_service's multi-GPU mode.

The reference scales gpu_service by running ``workers`` copies of one process on one device
(/root/reference/gpu_service/gunicorn_conf.py:9), each with its own model copy, and keeps vectors in
PostgreSQL (/root/reference/assistant/rag/services/search_service.py:185-196).  Here the W GPUs of a
node form ONE service: one process per GPU, RCCL (xGMI) for the data plane, gloo groups for the
host-side control plane.  The layout comes from the settings (``assistant.conf``):

* ``INDEX_SHARDS`` = S -- ranks 0..S-1 each hold a ``ShardedIndex`` shard (rows by ``id % S``);
  searches scan all shards and gather the partial top-k to rank 0 (12 B per hit).
* ``EMBED_DP`` = D     -- ranks 0..D-1 hold an encoder replica; a large ``/embeddings/`` batch (ingest)
  is split D ways (each rank receives only its texts) and the vectors are gathered to rank 0.
  Document ingest (``/index/{name}/ingest``) is rank-local instead: each text goes to the encoder
  rank that owns its row's shard, which embeds it and writes its shard from HBM.
* ``GEN_TP`` = T       -- W / T generator replicas; replica g is the TP group of ranks gT..gT+T-1.

(0 for S or D means "every rank".)  Rank 0 serves HTTP.  Two independent control channels:

* **Commands** (index upsert / delete / search / sizes, DP embedding): rank 0 broadcasts an int64
  header on the node's control group and moves the payload as typed tensors -- an upsert sends each
  shard only the rows it owns, an embedding batch sends each encoder rank only its texts.  Every
  rank runs the op in one order, so the RCCL collectives inside line up.  Followers run these on
  their main thread (``Node.follow``) and on a side HIP stream.
* **Generation**: every replica steps on its own.  Rank 0 places a request on the least-loaded
  replica and ships it over that replica's request link (a gloo pair group, one per direction) as a
  fixed-shape message (``parallel/wire.py``); the replica's leader (TP rank 0) runs its engine loop
  in a thread of its own and sends each finished output back when it finishes.  Inside a TP group
  the leader broadcasts the step's adds / aborts (and which models to step) to its peers: lock-step
  only within the group.  A search or an upsert therefore never waits behind a decode step.

Facades on rank 0 give the serving layer the single-process APIs it already uses:
``NodeLLM`` (the ``LLMEngine`` API under ``LLMWorker``), ``NodeEmbedder`` (the ``EmbeddingEngine``
API under ``EmbedWorker``) and ``NodeIndexes`` (gpu_service's ``/index/*`` backend, which validates
every payload before it becomes a command: a malformed request is a 400, not a broken group).

Failure model: a follower whose command or engine loop raises exits non-zero; rank
0 sees the broken link or collective, marks the node unhealthy (``/health`` 503) and its watchdog
exits, so the launcher (``torch.distributed.run --max-restarts``) restarts the whole group with new
RCCL communicators.  The index is a cache of the ORM and is reloaded from its snapshot / the DB.
"""
from __future__ import annotations

import itertools
import logging
import math
import queue
import threading
import time
from contextlib import nullcontext
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from .dist import force_group
from . import wire

logger = logging.getLogger(__name__)


class NodeFault(RuntimeError):
    """A node command failed: a rank died or a collective broke.  The group is unusable until the
    launcher restarts it (new process group, new RCCL communicators)."""


@dataclass
class NodePlan:
    world: int
    index_shards: int = 0
    embed_dp: int = 0
    gen_tp: int = 1

    def __post_init__(self):
        W = self.world
        self.index_shards = W if self.index_shards <= 0 else self.index_shards
        self.embed_dp = W if self.embed_dp <= 0 else self.embed_dp
        if not 1 <= self.index_shards <= W:
            raise ValueError(f"INDEX_SHARDS={self.index_shards} must be in [1, {W}]")
        if not 1 <= self.embed_dp <= W:
            raise ValueError(f"EMBED_DP={self.embed_dp} must be in [1, {W}]")
        if self.gen_tp < 1 or W % self.gen_tp:
            raise ValueError(f"GEN_TP={self.gen_tp} must divide the node's {W} ranks")

    @property
    def gen_replicas(self) -> int:
        return self.world // self.gen_tp

    @classmethod
    def from_settings(cls, world: int) -> "NodePlan":
        from ..engine.serving import setting

        return cls(world, index_shards=setting("INDEX_SHARDS", 0), embed_dp=setting("EMBED_DP", 0),
                   gen_tp=setting("GEN_TP", 1))


def _subgroup(n: int, world: int):
    """Ranks 0..n-1 as a group (None = the default group when it is everyone).  Collective."""
    return None if n == world else dist.new_group(list(range(n)))


# command op codes (header word 0 of the control broadcast)
_OPS = ("stop", "name", "index_upsert", "index_delete", "index_search", "index_sizes", "embed", "fault", "stats",
        "index_ingest")
_CODE = {op: i for i, op in enumerate(_OPS)}
_NORM = {None: -1, False: 0, True: 1}


def _i64(a) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.int64)))


def _texts_words(texts) -> tuple[np.ndarray, np.ndarray]:
    blobs = [t.encode("utf-8") for t in texts]
    offs = np.zeros(len(blobs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(b) for b in blobs])
    return offs, np.frombuffer(b"".join(blobs), dtype=np.uint8).astype(np.int64)


def _words_texts(offs, flat) -> list:
    raw = bytes(np.asarray(flat, dtype=np.int64).astype(np.uint8).tolist())
    return [raw[int(offs[i]):int(offs[i + 1])].decode("utf-8") for i in range(len(offs) - 1)]


class Node:
    """Per-rank state of the node service.  Constructed on every rank (collective: creates groups and
    engines in one order)."""

    def __init__(self, info, plan: NodePlan, embedders=(), providers=(), seed: int = 0, llm_kwargs=None,
                 embed_kwargs=None, ctrl=None, llm_weights=None):
        from . import dist as pdist
        from .tp_serving import control_group

        self.info, self.plan = info, plan
        self.rank, self.world = info.rank, info.world_size
        # commands go through the control group whenever one exists: W > 1, or a world-1 group
        # formed on purpose (DAB_FORCE_GROUP) so the broadcast paths run on one GPU too
        self.grouped = pdist.grouped()
        self.device = info.device
        assert plan.world == self.world, "plan built for another world size"
        W, T, R = self.world, plan.gen_tp, plan.gen_replicas
        if ctrl is None and self.grouped:
            ctrl = control_group(list(range(W)))
        self.ctrl = ctrl
        self.tp_group, self.tp_rank, self.replica = pdist.tp_groups(T)
        self.index_group = _subgroup(plan.index_shards, W)
        self.embed_group = _subgroup(plan.embed_dp, W)
        self.in_index = self.rank < plan.index_shards
        self.in_embed = self.rank < plan.embed_dp
        self.leader = self.replica * T  # global rank of this replica's TP rank 0
        # request links rank 0 <-> leader of replica g >= 1, one pair group per direction (each used
        # by one thread per side); TP control groups for the lock-step inside a replica
        self._down: dict = {}
        self._up: dict = {}
        for g in range(1, R):
            dn, up = control_group([0, g * T]), control_group([0, g * T])
            if self.rank in (0, g * T):
                self._down[g], self._up[g] = dn, up
        self.tp_ctrl = None
        if T > 1:
            for g in range(R):
                grp = control_group(list(range(g * T, (g + 1) * T)))
                if self.replica == g:
                    self.tp_ctrl = grp
        if T > 1 and len(providers) > 1:
            raise ValueError("GEN_TP > 1 serves one generator model per node")
        self.llms: dict = {}
        self.embeds: dict = {}
        self.indexes: dict = {}
        self.model_names = [p.lower() for p in providers]
        self.embed_names = [e.lower() for e in embedders]
        self.names: list[str] = []  # index names by id (same order on every rank)
        self._cmd_lock = threading.Lock()
        self._stopped = False
        self.commands = 0
        self.healthy = True
        self.last_error = ""
        self.stats = {"upsert_bytes_recv": 0, "embed_bytes_recv": 0, "ingest_bytes_recv": 0,
                      "ingest_vec_bytes_recv": 0, "ctrl_s": 0.0, "llm_steps": 0,
                      "link_bytes_sent": 0}
        self._side = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self._llm_thread: threading.Thread | None = None
        self._receivers: list[threading.Thread] = []
        self._outq: dict[int, queue.Queue] = {m: queue.Queue() for m in range(len(self.model_names))}
        from ..engine.embedding_engine import EmbeddingEngine
        from ..engine.llm_engine import LLMEngine

        for name in embedders:
            if self.in_embed:
                self.embeds[name.lower()] = EmbeddingEngine(name, self.device, seed=seed, **(embed_kwargs or {}))
        for name in providers:
            kw = dict(llm_kwargs or {})
            if llm_weights is not None:  # callable (name, tp_rank, tp_size) -> this rank's shard
                kw["weights"] = llm_weights(name, self.tp_rank, T)
            eng = LLMEngine(name, self.device, seed=seed, tp_group=self.tp_group, tp_size=T,
                            tp_rank=self.tp_rank, **kw)
            eng.auto_expire = False  # deadlines are decided on rank 0 and shipped as aborts
            self.llms[name.lower()] = eng

    # ================================================================== command channel
    def _side_stream(self):
        return torch.cuda.stream(self._side) if self._side is not None else nullcontext()

    def command(self, op: str, payload=None):
        """Rank 0: run ``op`` on every rank; returns rank 0's result."""
        assert self.rank == 0, "only rank 0 issues node commands"
        with self._cmd_lock:
            if self._stopped:
                raise RuntimeError("node service is shut down")
            if not self.healthy:
                raise NodeFault(f"node group is broken ({self.last_error}); waiting for the restart")
            try:
                if op in ("index_upsert", "index_delete", "index_search", "index_ingest") and \
                        payload[0] not in self.names:
                    self._run("name", payload[0])
                return self._run(op, payload)
            except Exception as exc:
                # A dead peer surfaces here: the control broadcast or a collective inside the op fails.
                # Results of a half-run command cannot be trusted on any rank, so the group is over.
                self.healthy = False
                self.last_error = f"{op}: {type(exc).__name__}: {exc}"
                logger.error("node command failed, group marked broken: %s", self.last_error)
                raise NodeFault(self.last_error) from exc

    def _run(self, op: str, payload):
        words = getattr(self, "_hdr_" + op)(payload) if hasattr(self, "_hdr_" + op) else []
        hdr = torch.zeros(wire.HDR, dtype=torch.int64)
        hdr[0] = _CODE[op]
        hdr[1:1 + len(words)] = torch.tensor(words, dtype=torch.int64)
        if self.grouped:
            dist.broadcast(hdr, src=0, group=self.ctrl)
        self.commands += 1
        with self._side_stream():
            out = getattr(self, "_op_" + op)(hdr.tolist(), payload)
        if self._side is not None:
            self._side.synchronize()
        return out

    def follow(self) -> int:
        """Ranks 1..W-1: start this rank's generator loop, then run commands until ``stop``.  Returns
        the number of commands run.  A command that raises ends the loop with the exception (the
        launcher restarts the group)."""
        self._start_llm_loop()
        n = 0
        while True:
            hdr = torch.zeros(wire.HDR, dtype=torch.int64)
            dist.broadcast(hdr, src=0, group=self.ctrl)
            h = hdr.tolist()
            op = _OPS[h[0]]
            if op == "stop":
                break
            try:
                with self._side_stream():
                    getattr(self, "_op_" + op)(h, None)
                if self._side is not None:
                    self._side.synchronize()
            except Exception:
                logger.exception("rank %d: node command %s failed; leaving the group", self.rank, op)
                raise
            n += 1
        if self._llm_thread is not None:
            self._llm_thread.join(120)
        return n

    def shutdown(self) -> None:
        if self.rank == 0 and not self._stopped:
            self._stop_llm_links()
            with self._cmd_lock:
                if self.grouped and self.healthy:
                    try:
                        self._run("stop", None)
                    except Exception:
                        logger.exception("stop broadcast failed")
                self._stopped = True

    def _bcast(self, t: torch.Tensor) -> torch.Tensor:
        if self.grouped:
            dist.broadcast(t, src=0, group=self.ctrl)
        return t

    # ------------------------------------------------------------------ ops (run on every rank)
    def _op_stop(self, h, p):
        return None

    def _hdr_name(self, name):
        return [len(name.encode("utf-8"))]

    def _op_name(self, h, name):
        buf = _i64(wire.text_words(name)) if self.rank == 0 else torch.zeros(h[1], dtype=torch.int64)
        self.names.append(wire.words_text(self._bcast(buf).numpy()))

    def _op_fault(self, h, p):
        """Fault injection (tests): the given rank fails inside a command."""
        if self.rank == h[1]:
            raise RuntimeError(f"injected fault on rank {h[1]}")

    def _hdr_fault(self, rank):
        return [int(rank)]

    def _cdev(self, group):
        if not self.grouped:
            return self.device
        return self.device if dist.get_backend(group) == "nccl" else torch.device("cpu")

    def _index(self, name: str, dim: int | None = None):
        idx = self.indexes.get(name)
        if idx is None and dim is not None and self.in_index:
            from ..engine.serving import setting
            from .sharded_index import ShardedIndex

            dtype = getattr(torch, str(setting("INDEX_DTYPE", "bfloat16")))
            idx = self.indexes[name] = ShardedIndex(dim, self.device, group=self.index_group, dtype=dtype)
        return idx

    def _index_total(self, local: int) -> int:
        t = torch.tensor([local], dtype=torch.int64, device=self._cdev(self.index_group))
        if self.grouped:
            dist.all_reduce(t, group=self.index_group)
        return int(t.item())

    def _hdr_index_upsert(self, p):
        name, ids, vecs, docs, groups = p
        return [self.names.index(name), vecs.shape[1], int(docs is not None), int(groups is not None), len(ids)]

    def _op_index_upsert(self, h, p):
        """Rows are routed by owner (``id % S``): shard r receives exactly its rows, rank 0 keeps its own."""
        name, dim, has_docs, has_groups, n = self.names[h[1]], h[2], h[3], h[4], h[5]
        S = self.plan.index_shards
        counts = torch.zeros(S, dtype=torch.int64)
        if self.rank == 0:
            _, ids, vecs, docs, groups = p
            owner = ids % S
            sel = [np.nonzero(owner == r)[0] for r in range(S)]
            counts = _i64([len(s) for s in sel])
        self._bcast(counts)
        mine = None
        if self.rank == 0:
            for r in range(1, S):
                if int(counts[r]) == 0:
                    continue
                s = sel[r]
                ints = np.stack([ids[s], docs[s] if has_docs else np.zeros(len(s), np.int64),
                                 groups[s].astype(np.int64) if has_groups else np.zeros(len(s), np.int64)])
                dist.send(_i64(ints), dst=r, group=self.ctrl)
                dist.send(torch.from_numpy(np.ascontiguousarray(vecs[s])), dst=r, group=self.ctrl)
            s = sel[0]
            mine = (ids[s], vecs[s], docs[s] if has_docs else None, groups[s] if has_groups else None)
        elif self.in_index and int(counts[self.rank]):
            m = int(counts[self.rank])
            ints = torch.zeros((3, m), dtype=torch.int64)
            v = torch.zeros((m, dim), dtype=torch.float32)
            dist.recv(ints, src=0, group=self.ctrl)
            dist.recv(v, src=0, group=self.ctrl)
            self.stats["upsert_bytes_recv"] += ints.numel() * 8 + v.numel() * 4
            a = ints.numpy()
            mine = (a[0], v.numpy(), a[1] if has_docs else None, a[2].astype(np.int32) if has_groups else None)
        if not self.in_index:
            return None
        idx = self._index(name, dim)
        if mine is not None and len(mine[0]):
            idx.add(mine[0], torch.from_numpy(np.ascontiguousarray(mine[1])), doc_ids=mine[2], groups=mine[3])
        return self._index_total(len(idx.local))

    def _hdr_index_delete(self, p):
        name, ids = p
        return [self.names.index(name), len(ids)]

    def _op_index_delete(self, h, p):
        ids = _i64(p[1]) if self.rank == 0 else torch.zeros(h[2], dtype=torch.int64)
        ids = self._bcast(ids).numpy()
        if not self.in_index:
            return None
        idx = self._index(self.names[h[1]])
        return self._index_total(idx.remove(ids) if idx is not None else 0)

    def _hdr_index_search(self, p):
        name, q, k, groups, allowed, doc_lt = p
        total = sum(len(a) for a in allowed) if allowed is not None else 0
        return [self.names.index(name), q.shape[0], q.shape[1], int(k), int(groups is not None),
                int(allowed is not None), total, int(doc_lt is not None)]

    def _op_index_search(self, h, p):
        name, nq, dim, k, has_g, has_a, total, has_d = self.names[h[1]], h[2], h[3], h[4], h[5], h[6], h[7], h[8]
        if self.rank == 0:
            _, q, _, groups, allowed, doc_lt = p
            qt = torch.from_numpy(np.ascontiguousarray(q, dtype=np.float32))
        else:
            qt = torch.zeros((nq, dim), dtype=torch.float32)
        self._bcast(qt)
        groups_t = allowed_l = doc_t = None
        if has_g:
            groups_t = self._bcast(_i64(groups) if self.rank == 0 else torch.zeros(nq, dtype=torch.int64))
        if has_a:
            if self.rank == 0:
                offs = np.zeros(nq + 1, dtype=np.int64)
                offs[1:] = np.cumsum([len(a) for a in allowed])
                flat = np.concatenate([np.asarray(a, dtype=np.int64).reshape(-1) for a in allowed]) if total else \
                    np.zeros(0, dtype=np.int64)
                offs_t, flat_t = _i64(offs), _i64(flat)
            else:
                offs_t, flat_t = torch.zeros(nq + 1, dtype=torch.int64), torch.zeros(total, dtype=torch.int64)
            self._bcast(offs_t)
            if total:
                self._bcast(flat_t)
            o, f = offs_t.numpy(), flat_t.numpy()
            allowed_l = [f[o[i]:o[i + 1]] for i in range(nq)]
        if has_d:
            doc_t = self._bcast(_i64(doc_lt) if self.rank == 0 else torch.zeros(nq, dtype=torch.int64))
        if not self.in_index:
            return None
        idx = self._index(name)
        out = idx.search_replicated(qt.numpy(), k, q_groups=None if groups_t is None else groups_t.numpy(),
                                    allowed=allowed_l, doc_lt=None if doc_t is None else doc_t.numpy(), dst=0)
        return None if out is None else tuple(x.cpu() for x in out)

    def _hdr_index_sizes(self, names):
        return [len(names)]

    def _op_index_sizes(self, h, names):
        ids = _i64([self.names.index(n) if n in self.names else -1 for n in names]) if self.rank == 0 else \
            torch.zeros(h[1], dtype=torch.int64)
        ids = self._bcast(ids).tolist()
        if not self.in_index:
            return None
        totals = []
        for i in ids:
            idx = self.indexes.get(self.names[i]) if i >= 0 else None
            totals.append(self._index_total(len(idx.local) if idx is not None else 0))
        return dict(zip(names, totals)) if self.rank == 0 else None

    def _hdr_embed(self, p):
        name, texts, normalize = p
        return [self.embed_names.index(name), len(texts), _NORM[normalize]]

    def _op_embed(self, h, p):
        """Each encoder rank receives only its round-robin share of the texts; vectors are gathered."""
        name, n, norm = self.embed_names[h[1]], h[2], {-1: None, 0: False, 1: True}[h[3]]
        D = self.plan.embed_dp
        if not self.in_embed:
            return None
        if self.rank == 0:
            texts = p[1]
            for r in range(1, D):
                offs, flat = _texts_words(texts[r::D])
                dist.send(_i64([len(flat)]), dst=r, group=self.embed_ctrl_group())
                dist.send(_i64(offs), dst=r, group=self.embed_ctrl_group())
                if len(flat):
                    dist.send(_i64(flat), dst=r, group=self.embed_ctrl_group())
            mine = texts[0::D]
        else:
            ln = torch.zeros(1, dtype=torch.int64)
            dist.recv(ln, src=0, group=self.embed_ctrl_group())
            cnt = len(range(self.rank, n, D))
            offs = torch.zeros(cnt + 1, dtype=torch.int64)
            dist.recv(offs, src=0, group=self.embed_ctrl_group())
            flat = torch.zeros(int(ln), dtype=torch.int64)
            if int(ln):
                dist.recv(flat, src=0, group=self.embed_ctrl_group())
            self.stats["embed_bytes_recv"] += 8 * (1 + offs.numel() + flat.numel())
            mine = _words_texts(offs.numpy(), flat.numpy())
        eng = self.embeds[name]
        v = eng.embed(mine, normalize=norm, out_dtype=torch.float32)
        if D == 1 and not force_group():  # one embedder: its vectors are the answer (no gather)
            return v
        cdev = self._cdev(self.embed_group)
        rows = math.ceil(n / D)
        buf = torch.zeros((rows, eng.dim), dtype=torch.float32, device=cdev)
        buf[: len(mine)] = v.to(cdev)
        parts = [torch.empty_like(buf) for _ in range(D)] if self.rank == 0 else None
        dist.gather(buf, parts, dst=0, group=self.embed_group)
        if self.rank != 0:
            return None
        out = torch.empty((n, eng.dim), dtype=torch.float32, device=cdev)
        for r in range(D):
            cnt = len(range(r, n, D))
            out[r::D] = parts[r][:cnt]
        return out

    def embed_ctrl_group(self):
        return self.ctrl

    # ------------------------------------------------------------------ rank-local ingest
    def _ingest_plan(self, ids) -> np.ndarray:
        """Encoder rank of each row: the shard owner itself when it holds an encoder (the default
        layout, S = D = W), else owner % D (the vectors of those rows then move to their owner)."""
        owner = np.asarray(ids, dtype=np.int64) % self.plan.index_shards
        return np.where(owner < self.plan.embed_dp, owner, owner % self.plan.embed_dp)

    def _hdr_index_ingest(self, p):
        name, model, ids, texts, docs, groups, normalize, ret = p
        dim = self.embeds[model].dim
        return [self.names.index(name), self.embed_names.index(model), len(ids), int(docs is not None),
                int(groups is not None), _NORM[normalize], int(ret), dim]

    def _op_index_ingest(self, h, p):
        """Embed + index write where the row lives: rank 0 routes each text (not a vector) to the
        encoder rank that owns the row's shard (``id % S``); that rank embeds its texts and adds
        the vectors to its own shard from HBM.  With the default layout no vector crosses a link;
        only the per-(encoder, owner) counts are broadcast and the new index size is reduced.
        ``ret`` gathers the vectors to rank 0 as well (for callers that store them in the DB, as
        the reference's embedding step does: assistant/processing/documents/steps/embeddings.py)."""
        name, model, n, has_docs, has_groups = self.names[h[1]], self.embed_names[h[2]], h[3], h[4], h[5]
        norm, ret, dim = {-1: None, 0: False, 1: True}[h[6]], h[7], h[8]
        S, D = self.plan.index_shards, self.plan.embed_dp
        cnt = torch.zeros((D, S), dtype=torch.int64)
        if self.rank == 0:
            _, _, ids, texts, docs, groups, _, _ = p
            enc = self._ingest_plan(ids)
            owner = ids % S
            # rows grouped by (encoder, owner): each encoder's share is contiguous per owner
            order = np.lexsort((owner, enc))
            np.add.at(cnt.numpy(), (enc, owner), 1)
        self._bcast(cnt)
        c = cnt.numpy()
        g = self.embed_ctrl_group()
        mine_ints = mine_texts = None
        if self.rank == 0:
            start = np.concatenate([[0], np.cumsum(c.sum(1))])
            for e in range(D):
                rows = order[start[e]:start[e + 1]]
                ints = np.stack([ids[rows], docs[rows] if has_docs else np.zeros(len(rows), np.int64),
                                 groups[rows].astype(np.int64) if has_groups else np.zeros(len(rows), np.int64)])
                tx = [texts[i] for i in rows]
                if e == 0:
                    mine_ints, mine_texts = ints, tx
                    continue
                if not len(rows):
                    continue
                offs, flat = _texts_words(tx)
                dist.send(_i64(ints), dst=e, group=g)
                dist.send(_i64(offs), dst=e, group=g)
                dist.send(_i64([len(flat)]), dst=e, group=g)
                if len(flat):
                    dist.send(_i64(flat), dst=e, group=g)
        elif self.in_embed and c[self.rank].sum():
            m = int(c[self.rank].sum())
            ints, offs, ln = torch.zeros((3, m), dtype=torch.int64), torch.zeros(m + 1, dtype=torch.int64), \
                torch.zeros(1, dtype=torch.int64)
            dist.recv(ints, src=0, group=g)
            dist.recv(offs, src=0, group=g)
            dist.recv(ln, src=0, group=g)
            flat = torch.zeros(int(ln), dtype=torch.int64)
            if int(ln):
                dist.recv(flat, src=0, group=g)
            self.stats["ingest_bytes_recv"] += 8 * (ints.numel() + offs.numel() + 1 + flat.numel())
            mine_ints, mine_texts = ints.numpy(), _words_texts(offs.numpy(), flat.numpy())
        vecs = None
        if self.in_embed and mine_texts:
            vecs = self.embeds[model].embed(mine_texts, normalize=norm, out_dtype=torch.float32)
        # index writes: own rows from HBM; rows of encoder-less shards (owner >= D) travel once
        if self.in_index:
            idx = self._index(name, dim)
            if self.rank < D and vecs is not None:
                lo = int(c[self.rank, :self.rank].sum())
                k = int(c[self.rank, self.rank])
                if k:
                    a = mine_ints[:, lo:lo + k]
                    idx.add(a[0], vecs[lo:lo + k], a[1] if has_docs else None,
                            a[2].astype(np.int32) if has_groups else None)
        for owner in range(D, S):
            src = owner % D
            k = int(c[src, owner])
            if not k:
                continue
            if self.rank == src:
                lo = int(c[src, :owner].sum())
                dist.send(_i64(mine_ints[:, lo:lo + k]), dst=owner, group=g)
                dist.send(vecs[lo:lo + k].cpu().contiguous(), dst=owner, group=g)
            elif self.rank == owner:
                ints, v = torch.zeros((3, k), dtype=torch.int64), torch.zeros((k, dim), dtype=torch.float32)
                dist.recv(ints, src=src, group=g)
                dist.recv(v, src=src, group=g)
                self.stats["ingest_vec_bytes_recv"] += v.numel() * 4
                a = ints.numpy()
                self._index(name, dim).add(a[0], v, a[1] if has_docs else None,
                                           a[2].astype(np.int32) if has_groups else None)
        total = self._index_total(len(self._index(name, dim).local)) if self.in_index else None
        if not ret:
            return total
        # optional: vectors back to rank 0, in request order
        if self.rank == 0:
            out = torch.empty((n, dim), dtype=torch.float32)
            start = np.concatenate([[0], np.cumsum(c.sum(1))])
            if vecs is not None:
                out[torch.from_numpy(order[start[0]:start[1]])] = vecs.cpu()
            for e in range(1, D):
                m = int(c[e].sum())
                if m:
                    v = torch.zeros((m, dim), dtype=torch.float32)
                    dist.recv(v, src=e, group=g)
                    out[torch.from_numpy(order[start[e]:start[e + 1]])] = v
            return total, out
        if self.in_embed and vecs is not None:
            dist.send(vecs.cpu().contiguous(), dst=0, group=g)
        return None

    def _op_stats(self, h, p):
        """Per-rank control-plane counters gathered to rank 0: [ctrl_s, llm_steps, upsert bytes, embed bytes,
        ingest text bytes, ingest vector bytes] (bytes received by that rank)."""
        t = torch.tensor([self.stats["ctrl_s"], self.stats["llm_steps"], self.stats["upsert_bytes_recv"],
                          self.stats["embed_bytes_recv"], self.stats["ingest_bytes_recv"],
                          self.stats["ingest_vec_bytes_recv"]], dtype=torch.float64)
        if not self.grouped:
            return t[None]
        parts = [torch.zeros_like(t) for _ in range(self.world)] if self.rank == 0 else None
        dist.gather(t, parts, dst=0, group=self.ctrl)
        return torch.stack(parts) if self.rank == 0 else None

    # ================================================================== generation
    def _engines(self):
        return [self.llms[n] for n in self.model_names]

    def _start_llm_loop(self):
        """Followers: the replica leader's request loop, or a TP peer's lock-step loop."""
        if not self.model_names or self._llm_thread is not None:
            return
        if self.rank == self.leader and self.rank != 0:
            target = self._leader_loop
        elif self.rank != self.leader:
            target = self._peer_loop
        else:
            return
        self._llm_thread = threading.Thread(target=self._guard(target), name=f"node-llm-{self.rank}", daemon=True)
        self._llm_thread.start()

    def _guard(self, fn):
        def run():
            try:
                fn()
            except Exception as exc:
                self.healthy = False
                self.last_error = f"generator loop: {type(exc).__name__}: {exc}"
                logger.exception("rank %d: generator loop failed; leaving the group", self.rank)
                import os

                os._exit(1)  # the launcher restarts the group
        return run

    def apply_items(self, items, outs: list | None) -> tuple[list, bool]:
        """Applies a batch of ADD / ABORT / FAIL / STOP items to the local engines.  Returns (models to
        step, stop); aborted requests' outputs are appended to ``outs`` (leaders) or dropped."""
        engines = self._engines()
        steps, stop = [], False
        for h, p in items:
            k = int(h[0])
            if k == wire.ADD:
                m, rid, prompt, sp = wire.read_add(h, p)
                try:
                    engines[m].add_request(prompt, sp, request_id=rid)
                except Exception as exc:  # a request the engine refuses fails alone, on every TP rank alike
                    logger.warning("rank %d: request %d refused: %s", self.rank, rid, exc)
                    if outs is not None:
                        outs.append(wire.out_item(m, engines[m].rejected_output(rid, prompt, str(exc))))
            elif k == wire.ABORT:
                m, rid, reason = wire.read_abort(h, p)
                if engines[m].abort(rid, reason):
                    out = engines[m].pop_output(rid)
                    if outs is not None:
                        outs.append(wire.out_item(m, out))
            elif k == wire.FAIL:
                engines[int(h[1])].fail_all()
            elif k == wire.STEP:
                steps.append(int(h[1]))
            elif k == wire.STOP:
                stop = True
        return steps, stop

    def step_models(self, steps, outs: list | None) -> None:
        engines = self._engines()
        for m in steps:
            for rid in engines[m].step():
                out = engines[m].pop_output(rid)
                if outs is not None:
                    outs.append(wire.out_item(m, out))
        self.stats["llm_steps"] += 1 if steps else 0

    def _leader_loop(self):
        """Leader of replica g >= 1: requests arrive on the down link (polled between steps, waited
        for when idle), outputs leave on the up link as they finish."""
        g = self.replica
        down, up = self._down[g], self._up[g]
        engines = self._engines()
        meta = torch.zeros(2, dtype=torch.int64)
        work = dist.irecv(meta, src=0, group=down)
        while True:
            busy = any(e.has_unfinished() for e in engines)
            items = []
            if not busy:
                work.wait()  # idle: sleep until rank 0 sends work (not counted as control time)
            t0 = time.perf_counter()
            if not busy or work.is_completed():
                items = wire.recv_batch(0, down, meta)
                meta = torch.zeros(2, dtype=torch.int64)
                work = dist.irecv(meta, src=0, group=down)
            outs: list = []
            _, stop = self.apply_items(items, outs)
            steps = [] if stop else [m for m, e in enumerate(engines) if e.has_unfinished()]
            if self.tp_ctrl is not None and (items or steps):
                wire.bcast_batch(list(items) + [wire.item([wire.STEP, m]) for m in steps], self.rank, self.tp_ctrl)
            self.stats["ctrl_s"] += time.perf_counter() - t0
            if stop:
                self.stats["link_bytes_sent"] += wire.send_batch(outs + [wire.item([wire.STOP])], 0, up)
                return
            self.step_models(steps, outs)
            if outs:
                t0 = time.perf_counter()
                self.stats["link_bytes_sent"] += wire.send_batch(outs, 0, up)
                self.stats["ctrl_s"] += time.perf_counter() - t0

    def _peer_loop(self):
        """TP rank > 0: apply what the replica's leader broadcasts, step when it steps."""
        while True:
            items = wire.bcast_batch(None, self.leader, self.tp_ctrl)  # waits out the leader's idle time too
            steps, stop = self.apply_items(items, None)
            if stop:
                return
            self.step_models(steps, None)

    def _ensure_receivers(self):
        """Rank 0: one thread per remote replica collects its finished outputs."""
        if self.rank != 0 or self._receivers:
            return
        for g, up in self._up.items():
            t = threading.Thread(target=self._receive, args=(g, up), name=f"node-recv-{g}", daemon=True)
            t.start()
            self._receivers.append(t)

    def _receive(self, g, up):
        src = g * self.plan.gen_tp
        try:
            while True:
                for h, p in wire.recv_batch(src, up):
                    k = int(h[0])
                    if k == wire.STOP:
                        return
                    if k == wire.OUT:
                        m = int(h[1])
                        _, out = wire.read_out(h, p, self.llms[self.model_names[m]].tokenizer)
                        self._outq[m].put(out)
        except Exception as exc:
            if not self._stopped:
                self.healthy = False
                self.last_error = f"replica {g} link: {type(exc).__name__}: {exc}"
                logger.error("node replica link broken: %s", self.last_error)

    def send_items(self, g: int, items) -> None:
        """Rank 0: ship items to replica g's leader."""
        t0 = time.perf_counter()
        self.stats["link_bytes_sent"] += wire.send_batch(items, g * self.plan.gen_tp, self._down[g])
        self.stats["ctrl_s"] += time.perf_counter() - t0

    def _stop_llm_links(self):
        if not self.model_names:
            return
        for g in self._down:
            try:
                self.send_items(g, [wire.item([wire.STOP])])
            except Exception:
                logger.exception("stop to replica %d failed", g)
        for t in self._receivers:
            t.join(60)
        if self.tp_ctrl is not None and self.healthy:
            wire.bcast_batch([wire.item([wire.STOP])], 0, self.tp_ctrl)


# ---------------------------------------------------------------------- rank-0 facades
class NodeLLM:
    """``LLMEngine`` API over the node's generator replicas (what ``LLMWorker`` drives).  Replica 0 is
    this rank's engine, stepped in the caller's thread; the other replicas run on their own and their
    finished outputs arrive through ``Node``'s receiver threads."""

    def __init__(self, node: Node, name: str):
        self.node, self.name = node, name.lower()
        self.m = node.model_names.index(self.name)
        self.engine = node.llms[self.name]  # replica 0's engine (tokenizer, limits, stats)
        self._ids = itertools.count()
        self._local: list = []  # items for replica 0 (applied / broadcast at the next step)
        self._remote: dict[int, list] = {g: [] for g in range(1, node.plan.gen_replicas)}
        self._where: dict[int, int] = {}
        self._deadline: dict[int, float] = {}
        self._load = [0] * node.plan.gen_replicas
        self.finished: dict = {}
        self._discard: set = set()
        self.stats_node = {"steps": 0, "placed": [0] * node.plan.gen_replicas}
        node._ensure_receivers()

    def add_request(self, prompt_ids, params=None, request_id=None) -> int:
        from ..engine.llm_engine import SamplingParams

        params = params or SamplingParams()
        self.engine.check_params(params)  # a bad schema fails this caller here, not a replica's step
        rid = next(self._ids) if request_id is None else int(request_id)
        replica = min(range(len(self._load)), key=lambda g: (self._load[g], g))
        it = wire.add_item(self.m, rid, [int(t) for t in prompt_ids], params)
        (self._local if replica == 0 else self._remote[replica]).append(it)
        self._where[rid] = replica
        self._load[replica] += 1
        self.stats_node["placed"][replica] += 1
        if params.timeout_s is not None:
            self._deadline[rid] = time.perf_counter() + params.timeout_s
        return rid

    def abort(self, rid: int, reason: str = "abort") -> bool:
        g = self._where.get(rid)
        if g is None:
            return False
        it = wire.abort_item(self.m, rid, reason)
        (self._local if g == 0 else self._remote[g]).append(it)
        return True

    def has_unfinished(self) -> bool:
        return bool(self._where) or bool(self._local) or any(self._remote.values())

    def expired(self) -> list[int]:
        now = time.perf_counter()
        return [rid for rid, t in self._deadline.items() if now > t]

    def step(self) -> list[int]:
        node = self.node
        for rid in self.expired():
            self._deadline.pop(rid, None)
            self.abort(rid, "timeout")
        for g, items in self._remote.items():
            if items:
                self._remote[g] = []
                node.send_items(g, items)
        outs: list = []
        items, self._local = self._local, []
        _, _ = node.apply_items(items, outs)
        steps = [self.m] if self.engine.has_unfinished() else []
        if node.tp_ctrl is not None and (items or steps):
            t0 = time.perf_counter()
            wire.bcast_batch(list(items) + [wire.item([wire.STEP, m]) for m in steps], 0, node.tp_ctrl)
            node.stats["ctrl_s"] += time.perf_counter() - t0
        node.step_models(steps, outs)
        self.stats_node["steps"] += 1
        got = [wire.read_out(h, p, self.engine.tokenizer)[1] for h, p in outs]
        q = node._outq[self.m]
        try:  # nothing ran here: wait briefly for a remote replica instead of spinning
            if not got and not steps:
                got.append(q.get(timeout=0.002))
            while True:
                got.append(q.get_nowait())
        except queue.Empty:
            pass
        done = []
        for out in got:
            rid = out.request_id
            g = self._where.pop(rid, None)
            if g is None:
                continue
            self._load[g] -= 1
            self._deadline.pop(rid, None)
            if rid in self._discard:
                self._discard.discard(rid)
                continue
            self.finished[rid] = out
            done.append(rid)
        return done

    def pop_output(self, rid: int):
        """The output of a finished request; for one still in flight (a cancelled caller) the output
        is dropped when it arrives and None is returned."""
        if rid in self.finished:
            return self.finished.pop(rid)
        if rid in self._where:
            self._discard.add(rid)
        return None

    def fail_all(self) -> list[int]:
        ids = list(self._where)
        node = self.node
        if node.healthy:  # a broken group is restarted as a whole; nothing to clean up remotely
            fail = [wire.item([wire.FAIL, self.m])]
            try:
                node.apply_items(fail, None)
                if node.tp_ctrl is not None:
                    wire.bcast_batch(fail, 0, node.tp_ctrl)
                for g in self._remote:
                    node.send_items(g, fail)
            except Exception:
                logger.exception("fail_all propagation failed")
        self._local.clear()
        for g in self._remote:
            self._remote[g] = []
        self._where.clear()
        self._deadline.clear()
        self._discard.clear()
        self._load = [0] * len(self._load)
        return ids

    def generate(self, prompts, params=None):
        """Batch helper with the ``LLMEngine.generate`` contract (tests, benchmarks)."""
        plist = params if isinstance(params, list) else [params] * len(prompts)
        rids = [self.add_request(self.engine.tokenizer.encode(p) if isinstance(p, str) else p, sp)
                for p, sp in zip(prompts, plist)]
        while self.has_unfinished():
            self.step()
        return [self.pop_output(r) for r in rids]

    @property
    def stats(self):
        return {**self.engine.stats, "node_steps": self.stats_node["steps"], "replicas": len(self._load),
                "in_flight": len(self._where)}

    def __getattr__(self, name):  # tokenizer, max_model_len, running, waiting, blocks ... of replica 0
        return getattr(self.engine, name)


class NodeEmbedder:
    """``EmbeddingEngine`` API (what ``EmbedWorker`` drives): batches of at least ``min_split``
    texts per rank are split over the ``EMBED_DP`` ranks, smaller ones run on rank 0 alone."""

    def __init__(self, node: Node, name: str, min_split: int = 32):
        self.node, self.name = node, name.lower()
        self.engine = node.embeds[self.name]
        self.min_split = min_split

    def embed(self, texts, normalize=None, out_dtype=torch.float32):
        texts = [str(t) for t in texts]
        D = self.node.plan.embed_dp
        if D == 1 or len(texts) < self.min_split * D:
            return self.engine.embed(texts, normalize=normalize, out_dtype=out_dtype)
        return self.node.command("embed", (self.name, texts, normalize)).to(out_dtype)

    def __getattr__(self, name):  # dim, cfg, stats, tokenize ...
        return getattr(self.engine, name)


class NodeIndexes:
    """gpu_service ``/index/*`` backend over the sharded index of the node.  Payloads are validated
    here, before they become commands: a malformed request raises ``ValueError`` (HTTP 400) and the
    group stays healthy."""

    MAX_K = 1024

    def __init__(self, node: Node):
        self.node = node
        self._dims: dict[str, int] = {}
        self._counts: dict[str, int] = {}

    def dim(self, name: str):
        return self._dims.get(name)

    def upsert(self, name, ids, vectors, doc_ids=None, groups=None) -> int:
        ids = np.asarray(ids)
        vecs = np.asarray(vectors, dtype=np.float32)
        if ids.ndim != 1 or (len(ids) and not np.issubdtype(ids.dtype, np.integer)):
            raise ValueError("ids must be a list of integers")
        ids = ids.astype(np.int64)
        if vecs.ndim != 2 or vecs.shape[0] != len(ids) or vecs.shape[1] < 1:
            raise ValueError("vectors must be a [len(ids), dim] matrix")
        if (ids < 0).any():
            raise ValueError("ids must be >= 0")
        if not np.isfinite(vecs).all():
            raise ValueError("vectors must be finite")
        dim = self._dims.get(name)
        if dim is not None and vecs.shape[1] != dim:
            raise ValueError(f"index {name} has dim {dim}")
        docs = None if doc_ids is None else np.asarray(doc_ids)
        if docs is not None and (docs.shape != ids.shape or (len(docs) and not np.issubdtype(docs.dtype, np.integer))):
            raise ValueError("doc_ids must be one integer per id")
        grp = None if groups is None else np.asarray(groups)
        if grp is not None:
            if grp.shape != ids.shape or (len(grp) and not np.issubdtype(grp.dtype, np.integer)):
                raise ValueError("groups must be one integer per id")
            if (grp < 0).any() or (grp >= 2 ** 31).any():
                raise ValueError("groups must be in [0, 2^31)")
        if len(ids) == 0:
            return self._counts.get(name, 0)
        self._dims.setdefault(name, vecs.shape[1])
        n = self.node.command("index_upsert", (name, ids, vecs, None if docs is None else docs.astype(np.int64),
                                               None if grp is None else grp.astype(np.int32)))
        self._counts[name] = n
        return n

    def ingest(self, name, model, ids, texts, doc_ids=None, groups=None, normalize=None,
               return_vectors=False):
        """Embed ``texts`` with ``model`` and upsert them as rows ``ids``, rank-locally (see
        ``Node._op_index_ingest``).  Returns the index size, or (size, [n, dim] vectors)."""
        model = str(model).lower()
        if model not in self.node.embed_names:
            raise ValueError(f"embedder {model} is not served")
        ids = np.asarray(ids)
        if ids.ndim != 1 or (len(ids) and not np.issubdtype(ids.dtype, np.integer)):
            raise ValueError("ids must be a list of integers")
        ids = ids.astype(np.int64)
        if (ids < 0).any():
            raise ValueError("ids must be >= 0")
        if len(texts) != len(ids) or not all(isinstance(t, str) for t in texts):
            raise ValueError("texts must hold one string per id")
        dim = self.node.embeds[model].dim
        if self._dims.get(name, dim) != dim:
            raise ValueError(f"index {name} has dim {self._dims[name]}, embedder {model} gives {dim}")
        docs = None if doc_ids is None else np.asarray(doc_ids)
        if docs is not None and (docs.shape != ids.shape or (len(docs) and not np.issubdtype(docs.dtype, np.integer))):
            raise ValueError("doc_ids must be one integer per id")
        grp = None if groups is None else np.asarray(groups)
        if grp is not None and (grp.shape != ids.shape or (len(grp) and not np.issubdtype(grp.dtype, np.integer))
                                or (grp < 0).any() or (grp >= 2 ** 31).any()):
            raise ValueError("groups must be one integer in [0, 2^31) per id")
        if len(ids) == 0:
            n = self._counts.get(name, 0)
            return (n, torch.zeros((0, dim))) if return_vectors else n
        self._dims.setdefault(name, dim)
        out = self.node.command("index_ingest", (name, model, ids, list(texts),
                                                 None if docs is None else docs.astype(np.int64),
                                                 None if grp is None else grp.astype(np.int32), normalize,
                                                 bool(return_vectors)))
        self._counts[name] = out[0] if return_vectors else out
        return out

    def delete(self, name, ids) -> int:
        if name not in self._dims:
            return 0
        ids = np.asarray(ids)
        if ids.ndim != 1 or (len(ids) and not np.issubdtype(ids.dtype, np.integer)):
            raise ValueError("ids must be a list of integers")
        before = self._counts.get(name, 0)
        n = self.node.command("index_delete", (name, ids.astype(np.int64)))
        self._counts[name] = before - n
        return n

    def size(self, name) -> int:
        return self._counts.get(name, 0)

    def search(self, name, queries, k, groups=None, allowed=None, doc_lt=None):
        if name not in self._dims:
            return None
        q = np.asarray(queries, dtype=np.float32)
        if q.ndim != 2 or q.shape[1] != self._dims[name]:
            raise ValueError(f"queries must be a [n, {self._dims[name]}] matrix")
        nq = q.shape[0]
        if not np.isfinite(q).all():
            raise ValueError("queries must be finite")
        k = int(k)
        if not 1 <= k <= self.MAX_K:
            raise ValueError(f"k must be in [1, {self.MAX_K}]")
        if groups is not None:
            groups = np.asarray(groups)
            if groups.shape != (nq,) or not np.issubdtype(groups.dtype, np.integer):
                raise ValueError("groups must be one integer per query")
        if allowed is not None:
            if len(allowed) != nq:
                raise ValueError("allowed must hold one id list per query")
            allowed = [np.asarray(list(a) if isinstance(a, (set, frozenset)) else a, dtype=np.int64).reshape(-1)
                       for a in allowed]
        if doc_lt is not None:
            doc_lt = np.asarray(doc_lt)
            if doc_lt.shape != (nq,) or not np.issubdtype(doc_lt.dtype, np.integer):
                raise ValueError("doc_lt must be one integer per query")
        return self.node.command("index_search", (name, q, k, groups, allowed, doc_lt))

    def sizes(self) -> dict:
        return dict(self._counts)
