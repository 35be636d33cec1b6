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

# Largest k one index search returns (the top-k kernels' bound; gpu_service rejects more with a 400)
MAX_SEARCH_K = 1024

SEARCHABLE = {
    "assistant_storage.question": "embedding",
    "assistant_storage.sentence": "embedding",
    "assistant_storage.document": "content_embedding",
}


def _key(model, field: str) -> str:
    return f"{model._meta.label_lower}.{field}"


def row_group(bot_id, completed) -> np.ndarray:
    """Row group the index kernels filter on: ``bot_id * 2 + completed`` (completed = the row's wiki
    has a COMPLETED processing run), so the reference's hot filter ``document__wiki__bot=B,
    document__wiki__processing__status=COMPLETED`` (steps/embeddings.py:26-29) is ONE group compare
    in the score epilogue -- no pk list, no mask."""
    b = np.asarray(bot_id, dtype=np.int64)
    return (b * 2 + np.asarray(completed, dtype=np.int64)).astype(np.int32)


def _completed_wikis() -> set:
    from assistant.storage.models import WikiDocumentProcessing

    return set(WikiDocumentProcessing.objects.filter(status=WikiDocumentProcessing.Status.COMPLETED)
               .values_list("wiki_document_id", flat=True))


def _meta_values(model, field, qs=None):
    """(ids, doc_ids, groups, vectors) of the rows with a non-null vector."""
    qs = model.objects.all() if qs is None else qs
    if model._meta.label_lower == "assistant_storage.document":
        rows = qs.exclude(**{f"{field}__isnull": True}).values_list("id", "id", "wiki__bot_id", "wiki_id", field)
    else:
        rows = qs.exclude(**{f"{field}__isnull": True}).values_list("id", "document_id", "document__wiki__bot_id",
                                                                     "document__wiki_id", field)
    ids, docs, bots, wikis, vecs = [], [], [], [], []
    for i, d, b, w, v in rows.iterator(chunk_size=4096):
        if v is None:
            continue
        ids.append(i)
        docs.append(d if d is not None else -1)
        bots.append(b if b is not None else 0)
        wikis.append(w if w is not None else -1)
        vecs.append(np.asarray(v, dtype=np.float32))
    dim = len(vecs[0]) if vecs else 0
    done = np.isin(np.asarray(wikis, dtype=np.int64), np.fromiter(_completed_wikis(), dtype=np.int64)) if ids else []
    return (np.asarray(ids, dtype=np.int64), np.asarray(docs, dtype=np.int64), row_group(bots, done),
            np.stack(vecs) if vecs else np.zeros((0, dim), dtype=np.float32))


# ------------------------------------------------------------------------------ QuerySet filter shapes

class IndexFilter:
    """A QuerySet filter the index evaluates itself: ``group`` (bot * 2 + completed), ``doc_lt``
    (document id bound), or ``all``.  ``None`` from ``index_filter_of`` = generic (pk allow-list)."""

    def __init__(self, group=None, doc_lt=None):
        self.group, self.doc_lt = group, doc_lt

    def __repr__(self):
        return f"IndexFilter(group={self.group}, doc_lt={self.doc_lt})"


HINT_ATTR = "_dab_index_filter"


def with_index_filter(qs, *, bot=None, completed=None, doc_lt=None):
    """Attach the filter the QuerySet encodes so the index can evaluate it without touching the DB.
    Used by the framework's own call sites; foreign QuerySets are recognised by ``index_filter_of``."""
    if bot is not None and completed:
        setattr(qs, HINT_ATTR, IndexFilter(group=int(row_group(getattr(bot, "pk", bot), 1))))
    elif doc_lt is not None and bot is None and completed is None:
        setattr(qs, HINT_ATTR, IndexFilter(doc_lt=int(doc_lt)))
    return qs


def index_filter_of(qs):
    """IndexFilter for a QuerySet the index can evaluate itself: the ``with_index_filter`` hint of the
    framework's own call sites (bot + COMPLETED group, reference steps/embeddings.py:26-29), an
    unfiltered QuerySet, or a document-id bound on the model's own table (reference processing
    steps/questions.py:121-126).  None for anything else (generic pk allow-list path).

    Filters that go through joins are never guessed from the WHERE tree: ``document__wiki__bot``
    looks like ``document__wiki__processing__...__bot`` or ``wiki__bot`` at the target field, so only
    the explicit hint selects the group path.  Hits are re-checked against the QuerySet by the caller
    (search_service loads them with ``qs.filter(pk__in=...)``), so the database stays authoritative
    even if a mirrored group bit is stale."""
    hint = getattr(qs, HINT_ATTR, None)
    if hint is not None:
        return hint
    where = qs.query.where
    if not where:
        return IndexFilter()
    try:
        return _recognise(qs, where)
    except Exception:  # unknown Django internals / lookups: generic path
        return None


def _base_alias(query):
    base = getattr(query, "base_table", None)
    if base is None:
        alias_map = getattr(query, "alias_map", None) or {}
        base = next(iter(alias_map), None)
    return base


def _recognise(qs, where):
    """Only a join-free ``<fk document>__lt`` / ``id__lt`` on the searched model's own table."""
    if where.negated or where.connector != "AND" or qs.query.low_mark or qs.query.high_mark is not None:
        return None
    if len(where.children) != 1:
        return None
    child = where.children[0]
    if not hasattr(child, "lhs") or not hasattr(child, "rhs") or child.lookup_name != "lt":
        return None
    alias = getattr(child.lhs, "alias", None)
    if alias is None or alias != _base_alias(qs.query):
        return None
    target = getattr(child.lhs, "target", None)
    if target is None:
        return None
    label, name = target.model._meta.label_lower, target.name
    if label != qs.model._meta.label_lower:
        return None
    if (label == "assistant_storage.document" and name == "id") or \
            (label in ("assistant_storage.question", "assistant_storage.sentence") and name == "document"):
        return IndexFilter(doc_lt=int(getattr(child.rhs, "pk", child.rhs)))
    return None


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

    def search(self, name, q, n, allowed, group, doc_lt=None):
        idx = self._idx.get(name)
        if idx is None or len(idx) == 0:
            return [], []
        sims, ids, _ = idx.search(np.asarray(q, dtype=np.float32)[None], min(n, MAX_SEARCH_K),
                                  q_groups=None if group is None else [group],
                                  allowed=None if allowed is None else [allowed],
                                  doc_lt=None if doc_lt is None else [doc_lt])
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

    def search(self, name, q, n, allowed, group, doc_lt=None):
        r = self._post(f"/index/{name}/search", {"queries": [list(map(float, q))], "k": min(int(n), MAX_SEARCH_K),
                                                 "groups": None if group is None else [int(group)],
                                                 "allowed": None if allowed is None else [list(map(int, allowed))],
                                                 "doc_lt": None if doc_lt is None else [int(doc_lt)]})
        return r["ids"][0], r["distances"][0]


class IndexService:
    def __init__(self, backend: str | None = None):
        self.backend_name = backend or settings.get("VECTOR_INDEX_BACKEND", None) or self._default_backend()
        self._lock = threading.RLock()
        self.stats = {"fast": 0, "generic": 0}
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

    def refresh_rows(self, model, pks, field="embedding"):
        """Re-mirror the given rows from the DB (current group bits / document ids); rows that no
        longer exist or lost their vector leave the index.  Called by a search whose hits the
        QuerySet rejected, i.e. whose mirrored metadata went stale."""
        if self._be is None:
            return
        name = _key(model, field)
        if not self._be.loaded(name):
            return
        pks = [int(p) for p in pks]
        ids, docs, groups, vecs = _meta_values(model, field, model.objects.filter(pk__in=pks))
        with self._lock:
            self._be.upsert(name, ids, vecs, docs, groups)
            gone = set(pks) - set(np.asarray(ids).tolist())
            if gone:
                self._be.remove(name, np.asarray(sorted(gone), dtype=np.int64))

    def refresh_wiki(self, wiki_id):
        """Re-mirror every searchable row of one wiki (finalize flips its completed bit and deletes the
        older runs' rows through the cascade)."""
        if self._be is None:
            return
        from assistant.storage.models import Document, Question, Sentence

        for model, field, flt in ((Question, "embedding", "document__wiki_id"),
                                  (Sentence, "embedding", "document__wiki_id"),
                                  (Document, "content_embedding", "wiki_id")):
            name = _key(model, field)
            if not self._be.loaded(name):
                continue
            ids, docs, groups, vecs = _meta_values(model, field, model.objects.filter(**{flt: wiki_id}))
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
        """Exact cosine search restricted to the QuerySet -> [(pk, distance)] ascending distance.

        The framework's two filter shapes (bot + COMPLETED, document id bound) and unfiltered
        QuerySets are evaluated inside the index (group compare / device mask; the group form keeps
        the threshold-search kernel); any other filter becomes a pk allow-list fetched with one
        ``values_list`` and mapped to rows vectorised."""
        model = qs.model
        q = np.asarray(query_embedding, dtype=np.float32)
        if self._be is None:
            return self._db_search(qs, q, n, field)
        self.ensure_loaded(model, field)
        flt = index_filter_of(qs)
        allowed = None
        if flt is None:
            allowed = np.fromiter(qs.values_list("pk", flat=True), dtype=np.int64)
            if not len(allowed):
                return []
            flt = IndexFilter()
        self.stats["fast" if allowed is None else "generic"] += 1
        ids, dist = self._be.search(_key(model, field), q, n, allowed, flt.group, flt.doc_lt)
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
