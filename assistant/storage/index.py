"""ORM <-> HBM vector-index bridge: the replacement of pgvector ``CosineDistance`` search.

Every embedding column that the framework searches (``Question.embedding``, ``Sentence.embedding``,
``Document.content_embedding``) is mirrored into an exact cosine top-k index.  Rows carry their
document id and bot id (the group the kernels filter on); arbitrary QuerySet filters become a per-query
allow-bitmask.  Backends (``settings.VECTOR_INDEX_BACKEND``):

  * ``engine``      -- in-process ``django_assistant_bot_amd.engine.vector_index.VectorIndex`` on the
                       local MI355X (CPU tensors when no GPU): fused MFMA score GEMM + radix top-k;
  * ``gpu_service`` -- the same index hosted by gpu_service (``/index/<name>/...`` endpoints), shared
                       by all web / Celery processes (sharded across the node's GPUs there);
  * ``db``          -- brute-force cosine in numpy over the rows of the QuerySet (config 1 of
                       BASELINE.json: CPU plumbing, ~1k documents).

The database stays the source of truth: indexes are (re)built lazily from it on first use, updated by
signals / explicit upserts after ``bulk_update``, and can be rebuilt with ``manage.py index_rebuild``.
"""
from __future__ import annotations

import json
import logging
import threading
import urllib.request

import numpy as np

from assistant.conf import settings

logger = logging.getLogger(__name__)

SEARCHABLE = {
    "assistant_storage.question": "embedding",
    "assistant_storage.sentence": "embedding",
    "assistant_storage.document": "content_embedding",
}


def _key(model, field: str) -> str:
    return f"{model._meta.label_lower}.{field}"


def _meta_values(model, field, qs=None):
    """(ids, doc_ids, groups, vectors) of the rows with a non-null vector."""
    qs = model.objects.all() if qs is None else qs
    if model._meta.label_lower == "assistant_storage.document":
        rows = qs.exclude(**{f"{field}__isnull": True}).values_list("id", "id", "wiki__bot_id", field)
    else:
        rows = qs.exclude(**{f"{field}__isnull": True}).values_list("id", "document_id", "document__wiki__bot_id",
                                                                     field)
    ids, docs, groups, vecs = [], [], [], []
    for i, d, g, v in rows.iterator(chunk_size=4096):
        if v is None:
            continue
        ids.append(i)
        docs.append(d if d is not None else -1)
        groups.append(g if g is not None else 0)
        vecs.append(np.asarray(v, dtype=np.float32))
    dim = len(vecs[0]) if vecs else 0
    return (np.asarray(ids, dtype=np.int64), np.asarray(docs, dtype=np.int64), np.asarray(groups, dtype=np.int32),
            np.stack(vecs) if vecs else np.zeros((0, dim), dtype=np.float32))


class _EngineBackend:
    def __init__(self):
        self._idx = {}

    def _get(self, name, dim):
        idx = self._idx.get(name)
        if idx is None:
            from django_assistant_bot_amd.engine.vector_index import VectorIndex

            idx = self._idx[name] = VectorIndex(dim)
        return idx

    def loaded(self, name):
        return name in self._idx

    def upsert(self, name, ids, vecs, docs, groups):
        if len(ids):
            self._get(name, vecs.shape[1]).add(ids, vecs, docs, groups)

    def remove(self, name, ids):
        if name in self._idx:
            self._idx[name].remove(ids)

    def search(self, name, q, n, allowed, group):
        idx = self._idx.get(name)
        if idx is None or len(idx) == 0:
            return [], []
        sims, ids, _ = idx.search(np.asarray(q, dtype=np.float32)[None], min(n, 1024),
                                  q_groups=None if group is None else [group],
                                  allowed=None if allowed is None else [set(allowed)])
        sims, ids = sims[0].float().cpu().numpy(), ids[0].cpu().numpy()
        keep = ids >= 0
        return ids[keep].tolist(), (1.0 - sims[keep]).tolist()


class _GPUServiceBackend:
    """Index hosted in gpu_service; synchronous JSON calls (signals and ORM code paths are sync)."""

    def __init__(self, base):
        self.base = base.rstrip("/")
        self._loaded = set()

    def _post(self, path, body):
        req = urllib.request.Request(f"{self.base}{path}", data=json.dumps(body).encode(),
                                     headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=120) as r:
            return json.loads(r.read() or b"{}")

    def loaded(self, name):
        return name in self._loaded

    def upsert(self, name, ids, vecs, docs, groups):
        self._loaded.add(name)
        if len(ids):
            self._post(f"/index/{name}/upsert", {"ids": ids.tolist(), "vectors": vecs.tolist(),
                                                 "doc_ids": docs.tolist(), "groups": groups.tolist()})

    def remove(self, name, ids):
        self._post(f"/index/{name}/delete", {"ids": list(map(int, ids))})

    def search(self, name, q, n, allowed, group):
        r = self._post(f"/index/{name}/search", {"queries": [list(map(float, q))], "k": int(n),
                                                 "groups": None if group is None else [int(group)],
                                                 "allowed": None if allowed is None else [list(map(int, allowed))]})
        return r["ids"][0], r["distances"][0]


class IndexService:
    def __init__(self, backend: str | None = None):
        self.backend_name = backend or settings.get("VECTOR_INDEX_BACKEND", None) or self._default_backend()
        self._lock = threading.RLock()
        if self.backend_name == "engine":
            self._be = _EngineBackend()
        elif self.backend_name == "gpu_service":
            self._be = _GPUServiceBackend(settings.GPU_SERVICE_ENDPOINT)
        elif self.backend_name == "db":
            self._be = None
        else:
            raise ValueError(f"unknown VECTOR_INDEX_BACKEND {self.backend_name}")

    @staticmethod
    def _default_backend():
        try:
            import django_assistant_bot_amd.engine.vector_index  # noqa: F401

            return "engine"
        except Exception:
            return "db"

    # ---------------------------------------------------------------- maintenance
    def ensure_loaded(self, model, field):
        if self._be is None:
            return
        name = _key(model, field)
        with self._lock:
            if not self._be.loaded(name):
                ids, docs, groups, vecs = _meta_values(model, field)
                logger.info("loading %d rows into index %s", len(ids), name)
                if len(ids):
                    self._be.upsert(name, ids, vecs, docs, groups)
                elif isinstance(self._be, _GPUServiceBackend):
                    self._be._loaded.add(name)

    def rebuild(self, model, field):
        if self._be is None:
            return 0
        name = _key(model, field)
        with self._lock:
            if isinstance(self._be, _EngineBackend):
                self._be._idx.pop(name, None)
            else:
                self._be._loaded.discard(name)
            self.ensure_loaded(model, field)
        return model.objects.exclude(**{f"{field}__isnull": True}).count()

    def upsert_objects(self, model, objs, field="embedding"):
        """Mirror rows after ``bulk_update``/``save`` (signals do not fire for bulk operations)."""
        if self._be is None:
            return
        name = _key(model, field)
        if not self._be.loaded(name):
            return  # will be loaded from the DB on first search
        ids = [o.pk for o in objs if getattr(o, field, None) is not None]
        if not ids:
            return
        ids, docs, groups, vecs = _meta_values(model, field, model.objects.filter(pk__in=ids))
        with self._lock:
            self._be.upsert(name, ids, vecs, docs, groups)

    def remove(self, model, ids, field="embedding"):
        if self._be is None:
            return
        name = _key(model, field)
        if self._be.loaded(name):
            with self._lock:
                self._be.remove(name, np.asarray(list(ids), dtype=np.int64))

    # ---------------------------------------------------------------- search
    def search(self, qs, query_embedding, n: int, field: str = "embedding"):
        """Exact cosine search restricted to the QuerySet -> [(pk, distance)] ascending distance."""
        model = qs.model
        q = np.asarray(query_embedding, dtype=np.float32)
        if self._be is None:
            return self._db_search(qs, q, n, field)
        self.ensure_loaded(model, field)
        allowed = None
        if qs.query.where:  # any filter -> exact allow-list (unfiltered QuerySets scan everything)
            allowed = list(qs.values_list("pk", flat=True))
            if not allowed:
                return []
        ids, dist = self._be.search(_key(model, field), q, n, allowed, None)
        return list(zip(ids, dist))

    @staticmethod
    def _db_search(qs, q, n, field):
        ids, _, _, vecs = _meta_values(qs.model, field, qs)
        if not len(ids):
            return []
        qn = q / (np.linalg.norm(q) or 1.0)
        vn = vecs / np.maximum(np.linalg.norm(vecs, axis=1, keepdims=True), 1e-12)
        dist = 1.0 - vn @ qn
        k = min(n, len(ids))
        part = np.argpartition(dist, k - 1)[:k]
        order = part[np.lexsort((ids[part], dist[part]))]
        return [(int(ids[i]), float(dist[i])) for i in order]


_service: IndexService | None = None


def get_index_service() -> IndexService:
    global _service
    if _service is None:
        _service = IndexService()
    return _service


def set_index_service(service: IndexService | None) -> None:
    global _service
    _service = service
