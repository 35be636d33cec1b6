"""One engine process group over the GPUs of a node: gpu_service's multi-GPU mode.

The reference scales gpu_service by running ``workers`` copies of one process on one device
(/root/reference/gpu_service/gunicorn_conf.py:9), each with its own model copy, and keeps vectors in
PostgreSQL (/root/reference/assistant/rag/services/search_service.py:185-196).  Here the W GPUs of a
node form ONE service: one process per GPU, RCCL (xGMI) for the data plane, a gloo group for the
host-side control plane.  The layout comes from the settings (``assistant.conf``):

* ``INDEX_SHARDS`` = S -- ranks 0..S-1 each hold a ``ShardedIndex`` shard (rows by ``id % S``);
  searches scan all shards and gather the partial top-k to rank 0 (12 B per hit).
* ``EMBED_DP`` = D     -- ranks 0..D-1 hold an encoder replica; a large ``/embeddings/`` batch (ingest)
  is split D ways and the vectors are gathered to rank 0 over RCCL.
* ``GEN_TP`` = T       -- W / T generator replicas; replica g is the TP group of ranks gT..gT+T-1.
  Requests are placed on the least-loaded replica; every scheduler step runs on all replicas.

(0 for S or D means "every rank".)  Rank 0 serves HTTP.  Every operation that involves other ranks is
a *command*: rank 0 takes the node lock, broadcasts ``(op, payload)`` on the control group, and then
every rank -- rank 0 included -- runs ``Node.execute(op, payload)``, so the RCCL collectives inside
the ops are issued in one order everywhere.  Ranks 1..W-1 sit in ``Node.follow()``.

Facades on rank 0 give the serving layer the single-process APIs it already uses:
``NodeLLM`` (the ``LLMEngine`` API under ``LLMWorker``), ``NodeEmbedder`` (the ``EmbeddingEngine``
API under ``EmbedWorker``) and ``NodeIndexes`` (gpu_service's ``/index/*`` backend).

Failure model: a follower whose command raises leaves the loop and exits non-zero;
the launcher (``torch.distributed.run --max-restarts``) then tears the whole group down and restarts
it, which rebuilds every RCCL communicator.  The index is a cache of the ORM and is reloaded from its
snapshot / the DB after a restart.
"""
from __future__ import annotations

import itertools
import logging
import math
import threading
import time
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

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


class Node:
    """Per-rank state of the node service.  Constructed on every rank (collective: creates groups and
    engines in one order)."""

    def __init__(self, info, plan: NodePlan, embedders=(), providers=(), seed: int = 0, llm_kwargs=None,
                 embed_kwargs=None, ctrl=None, llm_weights=None):
        from . import dist as pdist
        from .tp_serving import control_group

        self.info, self.plan = info, plan
        self.rank, self.world = info.rank, info.world_size
        self.device = info.device
        assert plan.world == self.world, "plan built for another world size"
        if ctrl is None and self.world > 1:
            ctrl = control_group(list(range(self.world)))
        self.ctrl = ctrl
        self.tp_group, self.tp_rank, self.replica = pdist.tp_groups(plan.gen_tp)
        self.index_group = _subgroup(plan.index_shards, self.world)
        self.embed_group = _subgroup(plan.embed_dp, self.world)
        self.in_index = self.rank < plan.index_shards
        self.in_embed = self.rank < plan.embed_dp
        self.llms: dict = {}
        self.embeds: dict = {}
        self.indexes: dict = {}
        self._lock = threading.RLock()
        self._stopped = False
        self.commands = 0
        self.healthy = True
        self.last_error = ""
        from ..engine.embedding_engine import EmbeddingEngine
        from ..engine.llm_engine import LLMEngine

        for name in embedders:
            if self.in_embed:
                self.embeds[name.lower()] = EmbeddingEngine(name, self.device, seed=seed, **(embed_kwargs or {}))
        for name in providers:
            kw = dict(llm_kwargs or {})
            if llm_weights is not None:  # callable (name, tp_rank, tp_size) -> this rank's shard
                kw["weights"] = llm_weights(name, self.tp_rank, plan.gen_tp)
            eng = LLMEngine(name, self.device, seed=seed, tp_group=self.tp_group, tp_size=plan.gen_tp,
                            tp_rank=self.tp_rank, **kw)
            eng.auto_expire = False  # deadlines are decided on rank 0 and shipped as aborts
            self.llms[name.lower()] = eng

    # ------------------------------------------------------------------ control plane
    def command(self, op: str, payload=None):
        """Rank 0: run ``op`` on every rank; returns rank 0's result."""
        assert self.rank == 0, "only rank 0 issues node commands"
        with self._lock:
            if self._stopped:
                raise RuntimeError("node service is shut down")
            if not self.healthy:
                raise NodeFault(f"node group is broken ({self.last_error}); waiting for the restart")
            try:
                if self.world > 1:
                    dist.broadcast_object_list([(op, payload)], src=0, group=self.ctrl)
                self.commands += 1
                return self.execute(op, payload)
            except Exception as exc:
                # A dead peer surfaces here: the control broadcast or a collective inside the op fails.
                # Results of a half-run command cannot be trusted on any rank, so the group is over.
                self.healthy = False
                self.last_error = f"{op}: {type(exc).__name__}: {exc}"
                logger.error("node command failed, group marked broken: %s", self.last_error)
                raise NodeFault(self.last_error) from exc

    def follow(self) -> int:
        """Ranks 1..W-1: run commands until ``stop``.  Returns the number of commands run.  A command
        that raises ends the loop with the exception (the launcher restarts the group)."""
        n = 0
        while True:
            box = [None]
            dist.broadcast_object_list(box, src=0, group=self.ctrl)
            op, payload = box[0]
            if op == "stop":
                return n
            try:
                self.execute(op, payload)
            except Exception:
                logger.exception("rank %d: node command %s failed; leaving the group", self.rank, op)
                raise
            n += 1

    def shutdown(self) -> None:
        if self.rank == 0 and not self._stopped:
            with self._lock:
                if self.world > 1:
                    dist.broadcast_object_list([("stop", None)], src=0, group=self.ctrl)
                self._stopped = True

    def execute(self, op: str, payload):
        return getattr(self, "_op_" + op)(payload)

    def _op_fault(self, rank):
        """Fault injection (tests): the given rank fails inside a command."""
        if self.rank == rank:
            raise RuntimeError(f"injected fault on rank {rank}")

    # ------------------------------------------------------------------ ops (run on every rank)
    def _cdev(self, group):
        if self.world == 1:
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
        if self.plan.index_shards > 1:
            dist.all_reduce(t, group=self.index_group)
        return int(t.item())

    def _op_index_upsert(self, p):
        name, ids, vecs, docs, groups = p
        if not self.in_index:
            return None
        idx = self._index(name, vecs.shape[1])
        idx.add(ids, torch.from_numpy(vecs), doc_ids=docs, groups=groups)
        return self._index_total(len(idx.local))

    def _op_index_delete(self, p):
        name, ids = p
        if not self.in_index:
            return None
        idx = self._index(name)
        return self._index_total(idx.remove(ids) if idx is not None else 0)

    def _op_index_search(self, p):
        name, queries, k, groups, allowed, doc_lt = p
        if not self.in_index:
            return None
        out = self._index(name).search_replicated(queries, k, q_groups=groups, allowed=allowed, doc_lt=doc_lt,
                                                  dst=0)
        return None if out is None else tuple(x.cpu() for x in out)

    def _op_index_sizes(self, names):
        if not self.in_index:
            return None
        return {n: self._index_total(len(self.indexes[n].local) if n in self.indexes else 0) for n in names}

    def _op_embed(self, p):
        name, texts, normalize = p
        if not self.in_embed:
            return None
        D = self.plan.embed_dp
        eng = self.embeds[name]
        n = len(texts)
        mine = texts[self.rank::D]  # round-robin: every rank gets a similar length mix
        v = eng.embed(mine, normalize=normalize, out_dtype=torch.float32)
        if D == 1:
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

    def _op_llm_step(self, p):
        name, items = p
        eng = self.llms[name]
        aborted = []
        for it in items:
            if it[1] != self.replica:
                continue
            if it[0] == "add":
                _, _, prompt, params, rid = it
                eng.add_request(prompt, params, request_id=rid)
            elif it[0] == "abort":
                _, _, rid, reason = it
                if eng.abort(rid, reason):
                    aborted.append(rid)
        done = eng.step() if eng.has_unfinished() else []
        outs = [(rid, eng.pop_output(rid)) for rid in aborted + done]
        if self.tp_rank != 0:
            outs = []  # the replica's TP rank 0 reports; the others only free their bookkeeping
        if self.world == 1:
            return outs
        got = [None] * self.world if self.rank == 0 else None
        dist.gather_object(outs, got, dst=0, group=self.ctrl)
        return [o for part in got for o in part] if self.rank == 0 else None

    def _op_llm_fail(self, name):
        return self.llms[name].fail_all()


# ---------------------------------------------------------------------- rank-0 facades
class NodeLLM:
    """``LLMEngine`` API over the node's generator replicas (what ``LLMWorker`` drives).  Adds and
    aborts are queued and shipped with the next step command; finished outputs come back from every
    replica's TP rank 0 in the same command."""

    def __init__(self, node: Node, name: str):
        self.node, self.name = node, name.lower()
        self.engine = node.llms[self.name]  # replica 0's engine (tokenizer, limits, stats)
        self._ids = itertools.count()
        self._pending: list = []
        self._where: dict[int, int] = {}
        self._deadline: dict[int, float] = {}
        self._load = [0] * node.plan.gen_replicas
        self.finished: dict = {}
        self._discard: set = set()
        self.stats_node = {"steps": 0, "placed": [0] * node.plan.gen_replicas}

    def add_request(self, prompt_ids, params=None, request_id=None) -> int:
        from ..engine.llm_engine import SamplingParams

        params = params or SamplingParams()
        rid = next(self._ids) if request_id is None else int(request_id)
        replica = min(range(len(self._load)), key=lambda g: (self._load[g], g))
        self._pending.append(("add", replica, [int(t) for t in prompt_ids], params, rid))
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
        self._pending.append(("abort", g, rid, reason))
        return True

    def has_unfinished(self) -> bool:
        return bool(self._where) or bool(self._pending)

    def expired(self) -> list[int]:
        now = time.perf_counter()
        return [rid for rid, t in self._deadline.items() if now > t]

    def step(self) -> list[int]:
        for rid in self.expired():
            self._deadline.pop(rid, None)
            self.abort(rid, "timeout")
        items, self._pending = self._pending, []
        outs = self.node.command("llm_step", (self.name, items))
        self.stats_node["steps"] += 1
        done = []
        for rid, out in outs:
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
        if self.node.healthy:  # a broken group is restarted as a whole; nothing to clean up remotely
            try:
                self.node.command("llm_fail", self.name)
            except NodeFault:
                pass
        self._pending.clear()
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
        texts = list(texts)
        D = self.node.plan.embed_dp
        if D == 1 or len(texts) < self.min_split * D:
            return self.engine.embed(texts, normalize=normalize, out_dtype=out_dtype)
        return self.node.command("embed", (self.name, texts, normalize)).to(out_dtype)

    def __getattr__(self, name):  # dim, cfg, stats, tokenize ...
        return getattr(self.engine, name)


class NodeIndexes:
    """gpu_service ``/index/*`` backend over the sharded index of the node."""

    def __init__(self, node: Node):
        self.node = node
        self._dims: dict[str, int] = {}
        self._counts: dict[str, int] = {}

    def dim(self, name: str):
        return self._dims.get(name)

    def upsert(self, name, ids, vectors, doc_ids=None, groups=None) -> int:
        vecs = np.asarray(vectors, dtype=np.float32)
        ids = np.asarray(ids, dtype=np.int64)
        docs = None if doc_ids is None else np.asarray(doc_ids, dtype=np.int64)
        grp = None if groups is None else np.asarray(groups, dtype=np.int32)
        self._dims.setdefault(name, vecs.shape[1])
        n = self.node.command("index_upsert", (name, ids, vecs, docs, grp))
        self._counts[name] = n
        return n

    def delete(self, name, ids) -> int:
        if name not in self._dims:
            return 0
        before = self._counts.get(name, 0)
        n = self.node.command("index_delete", (name, np.asarray(ids, dtype=np.int64)))
        self._counts[name] = before - n
        return n

    def size(self, name) -> int:
        return self._counts.get(name, 0)

    def search(self, name, queries, k, groups=None, allowed=None, doc_lt=None):
        if name not in self._dims:
            return None
        q = np.asarray(queries, dtype=np.float32)
        return self.node.command("index_search", (name, q, int(k), groups, allowed, doc_lt))

    def sizes(self) -> dict:
        return dict(self._counts)
