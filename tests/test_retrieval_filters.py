"""Filtered exact search: the index-side filters (group = bot*2 + completed, document-id bound,
vectorised pk allow-lists) against a brute-force oracle, and the ORM bridge's QuerySet-shape
recognition (reference steps/embeddings.py:26-29, processing steps/questions.py:121-126)."""
import types

import numpy as np
import pytest
import torch

from assistant.storage import index as index_mod
from django_assistant_bot_amd.engine.vector_index import VectorIndex

N, DIM = 3000, 64


@pytest.fixture(scope="module")
def data():
    rng = np.random.default_rng(0)
    vecs = rng.standard_normal((N, DIM)).astype(np.float32)
    ids = rng.permutation(10 * N)[:N].astype(np.int64) + 5
    docs = rng.integers(0, 400, N).astype(np.int64)
    bots = rng.integers(1, 4, N)
    done = rng.integers(0, 2, N)
    groups = index_mod.row_group(bots, done)
    return vecs, ids, docs, groups


def oracle(vecs, ids, q, k, keep):
    vn = vecs / np.linalg.norm(vecs, axis=1, keepdims=True)
    qn = q / np.linalg.norm(q)
    s = (torch.from_numpy(vn).to(torch.bfloat16).float().numpy() @
         torch.from_numpy(qn).to(torch.bfloat16).float().numpy())
    s = np.where(keep, s, -np.inf)
    order = np.argsort(-s, kind="stable")[:k]
    order = order[np.isfinite(s[order])]
    return set(ids[order].tolist()), s[order]


def build(data):
    vecs, ids, docs, groups = data
    idx = VectorIndex(DIM, device="cpu")
    idx.add(ids, vecs, doc_ids=docs, groups=groups)
    return idx


def check(idx, data, q, k, keep, **kw):
    vecs, ids, _, _ = data
    sims, got, _ = idx.search(q[None], k, **kw)
    got_ids = [i for i in got[0].tolist() if i >= 0]
    exp_ids, exp_s = oracle(vecs, ids, q, k, keep)
    assert len(got_ids) == len(exp_ids)
    # ties at the k-th score may swap members: compare scores, and ids away from the boundary
    np.testing.assert_allclose(np.sort(sims[0][: len(got_ids)].numpy())[::-1], np.sort(exp_s)[::-1], atol=1e-5)
    assert len(set(got_ids) ^ exp_ids) <= 2


@pytest.mark.parametrize("k", [1, 5, 250])
def test_group_filter_matches_oracle(data, k):
    idx = build(data)
    q = np.random.default_rng(k).standard_normal(DIM).astype(np.float32)
    g = int(index_mod.row_group(2, 1))
    check(idx, data, q, k, data[3] == g, q_groups=[g])


@pytest.mark.parametrize("bound", [0, 37, 200, 10_000])
def test_doc_lt_filter_matches_oracle(data, bound):
    idx = build(data)
    q = np.random.default_rng(bound).standard_normal(DIM).astype(np.float32)
    check(idx, data, q, 7, data[2] < bound, doc_lt=[bound])


def test_allow_list_array_and_set_match_oracle(data):
    idx = build(data)
    rng = np.random.default_rng(3)
    allowed = rng.choice(data[1], 500, replace=False)
    keep = np.isin(data[1], allowed)
    q = rng.standard_normal(DIM).astype(np.float32)
    check(idx, data, q, 20, keep, allowed=[allowed])
    check(idx, data, q, 20, keep, allowed=[set(allowed.tolist()) | {-99, 10 ** 9}])  # unknown ids ignored


def test_filters_compose_and_survive_deletes(data):
    idx = build(data)
    vecs, ids, docs, groups = data
    dead = ids[::7]
    idx.remove(dead)
    g = int(index_mod.row_group(1, 0))
    keep = (groups == g) & (docs < 250) & ~np.isin(ids, dead)
    q = np.random.default_rng(9).standard_normal(DIM).astype(np.float32)
    check(idx, data, q, 50, keep, q_groups=[g], doc_lt=[250])
    idx.compact()
    check(idx, data, q, 50, keep, q_groups=[g], doc_lt=[250])


def test_rows_of_is_vectorised_and_tracks_upserts(data):
    idx = build(data)
    ids = data[1]
    rows = idx.rows_of(ids[:10])
    assert rows.tolist() == [idx._row_of[int(i)] for i in ids[:10]]
    idx.add([123456789], np.ones((1, DIM), np.float32), doc_ids=[1], groups=[0])
    assert idx.rows_of([123456789]).tolist() == [idx._row_of[123456789]]
    idx.remove([123456789])
    assert idx.rows_of([123456789]).size == 0


# ------------------------------------------------------------------ ORM bridge with stub QuerySets

class _Meta:
    def __init__(self, label):
        self.label_lower = label


def _field(label, name):
    return types.SimpleNamespace(model=types.SimpleNamespace(_meta=_Meta(label)), name=name)


def _lookup(label, name, lookup, rhs, alias="T0"):
    """A WHERE-tree leaf as Django builds it: ``lhs`` is a Col with the table alias it reads."""
    return types.SimpleNamespace(lhs=types.SimpleNamespace(target=_field(label, name), alias=alias),
                                 lookup_name=lookup, rhs=rhs)


class _Where(list):
    negated = False
    connector = "AND"

    @property
    def children(self):
        return list(self)


class StubQS:
    def __init__(self, children, pks=()):
        self.model = types.SimpleNamespace(_meta=_Meta("assistant_storage.question"))
        self.query = types.SimpleNamespace(where=_Where(children), low_mark=0, high_mark=None, base_table="T0")
        self._pks = list(pks)
        self.values_list_calls = 0

    def values_list(self, *a, **kw):
        self.values_list_calls += 1
        return list(self._pks)


def test_recognises_only_join_free_document_bounds():
    """Join-free ``document__id__lt`` (ingest dedup) is evaluated in the index.  Filters through joins
    are never guessed from the WHERE tree (``document__wiki__bot`` and
    ``document__processing__status`` share target fields with the framework's hot filter but not its
    meaning): they take the pk allow-list path unless the call site attached the hint."""
    bot = types.SimpleNamespace(pk=3)
    hot = StubQS([_lookup("assistant_storage.wikidocument", "bot", "exact", bot, alias="T2"),
                  _lookup("assistant_storage.wikidocumentprocessing", "status", "exact", "completed", alias="T3")])
    assert index_mod.index_filter_of(hot) is None
    doc_status = StubQS([_lookup("assistant_storage.wikidocumentprocessing", "status", "exact", "completed",
                                 alias="T4")])
    assert index_mod.index_filter_of(doc_status) is None
    dedup = StubQS([_lookup("assistant_storage.question", "document", "lt", 41)])
    assert index_mod.index_filter_of(dedup).doc_lt == 41
    joined_lt = StubQS([_lookup("assistant_storage.question", "document", "lt", 41, alias="T7")])
    assert index_mod.index_filter_of(joined_lt) is None
    assert index_mod.index_filter_of(StubQS([])).group is None
    other = StubQS([_lookup("assistant_storage.question", "text", "icontains", "x")])
    assert index_mod.index_filter_of(other) is None


def test_hint_wins_over_recognition():
    qs = index_mod.with_index_filter(StubQS([_lookup("x", "y", "exact", 1)]), bot=5, completed=True)
    assert index_mod.index_filter_of(qs).group == int(index_mod.row_group(5, 1))


def test_service_fast_and_generic_paths_equal_oracle(data, monkeypatch):
    vecs, ids, docs, groups = data
    svc = index_mod.IndexService(backend="engine")
    svc._be.upsert("assistant_storage.question.embedding", ids, vecs, docs, groups)
    monkeypatch.setattr(svc, "ensure_loaded", lambda *a: None)
    q = np.random.default_rng(5).standard_normal(DIM).astype(np.float32)
    bot = 2
    hot = index_mod.with_index_filter(
        StubQS([_lookup("assistant_storage.wikidocument", "bot", "exact", bot, alias="T2"),
                _lookup("assistant_storage.wikidocumentprocessing", "status", "exact", "completed", alias="T3")]),
        bot=bot, completed=True)
    got = svc.search(hot, q, 250)
    assert hot.values_list_calls == 0 and svc.stats["fast"] == 1
    exp, _ = oracle(vecs, ids, q, 250, groups == index_mod.row_group(bot, 1))
    assert len(set(p for p, _ in got) ^ exp) <= 2
    assert all(a[1] <= b[1] + 1e-6 for a, b in zip(got, got[1:]))  # ascending distance
    # generic filter: one values_list, same answer as the oracle over the pk set
    allowed = ids[groups == index_mod.row_group(bot, 1)]
    gen = StubQS([_lookup("assistant_storage.question", "text", "icontains", "x")], pks=allowed.tolist())
    got2 = svc.search(gen, q, 250)
    assert gen.values_list_calls == 1 and svc.stats["generic"] == 1
    assert [p for p, _ in got2] == [p for p, _ in got]


class _Obj:
    def __init__(self, pk):
        self.pk = pk


class _FilterQS:
    """QuerySet stub whose ``filter(pk__in=...)`` applies its own membership (the DB's answer)."""

    def __init__(self, members):
        self.members = set(members)
        self.model = types.SimpleNamespace(objects=self)

    def filter(self, pk__in):
        return [_Obj(p) for p in pk__in if p in self.members]

    def in_bulk(self, pks):  # pragma: no cover - must not be used when filter works
        raise AssertionError("in_bulk bypasses the QuerySet filter")


def test_hits_are_rechecked_against_the_queryset():
    """A row the index returns but the QuerySet excludes (stale group bit) never reaches the caller."""
    from assistant.rag.services.search_service import _load_within

    got = _load_within(_FilterQS({1, 2, 5}), [5, 9, 1])
    assert sorted(got) == [1, 5]


def test_stale_group_bits_refill_to_n(data, monkeypatch):
    """LIMIT n semantics under a stale mirror: the index still files rows under bot 2 /
    COMPLETED that the DB has since moved elsewhere.  ``embedding_search_questions(..., n=5)`` drops
    them, re-mirrors them from the DB and searches again: 5 rows, the exact top 5 of the rows the
    QuerySet admits."""
    import asyncio

    from assistant.rag.services import search_service

    vecs, ids, docs, groups = data
    bot, g_hot = 2, int(index_mod.row_group(2, 1))
    q = np.random.default_rng(11).standard_normal(DIM).astype(np.float32)
    hot_rows = np.flatnonzero(groups == g_hot)
    order = [int(i) for i in ids[hot_rows][np.argsort(-(vecs[hot_rows] / np.linalg.norm(vecs[hot_rows], axis=1,
                                                                                      keepdims=True)) @ q)]]
    stale = set(order[:3])  # the 3 best mirrored rows no longer belong to the filter in the DB
    db_groups = {int(i): int(g) for i, g in zip(ids, groups)}
    for pk in stale:
        db_groups[pk] = int(index_mod.row_group(3, 1))

    svc = index_mod.IndexService(backend="engine")
    name = "assistant_storage.question.embedding"
    svc._be.upsert(name, ids, vecs, docs, groups)
    monkeypatch.setattr(svc, "ensure_loaded", lambda *a: None)
    row_of = {int(i): r for r, i in enumerate(ids)}

    def meta(model, field, rows):  # the DB's current view of the requested rows
        pks = np.asarray([o.pk for o in rows], dtype=np.int64)
        r = np.asarray([row_of[int(p)] for p in pks], dtype=np.int64)
        return pks, docs[r], np.asarray([db_groups[int(p)] for p in pks], dtype=np.int32), vecs[r]

    monkeypatch.setattr(index_mod, "_meta_values", meta)
    members = {pk for pk, g in db_groups.items() if g == g_hot}
    qs = index_mod.with_index_filter(StubQS([]), bot=bot, completed=True)
    fqs = _FilterQS(members)
    qs.filter, qs.model = fqs.filter, types.SimpleNamespace(_meta=_Meta("assistant_storage.question"), objects=fqs)
    monkeypatch.setattr(index_mod, "get_index_service", lambda: svc)
    got = asyncio.run(search_service.embedding_search_questions(q, qs, n=5))
    assert [o.pk for o in got] == order[3:8]
    assert all(a.distance <= b.distance + 1e-6 for a, b in zip(got, got[1:]))
    # the mirror is repaired: the next search needs no refill
    hits = svc.search(qs, q, 5)
    assert [p for p, _ in hits] == order[3:8]


def test_refill_never_asks_past_the_largest_k(data, monkeypatch):
    """``embedding_search`` asks for n = 10 * 10 * 10 = 1000 rows; a stale hit used to double
    the next request to >= 2000, which gpu_service rejects (k <= 1024, gpu_service/main.py) and the
    whole RAG search failed.  A backend with gpu_service's bound: every request stays <= 1024 and the
    search returns the qualifying rows."""
    import asyncio

    from assistant.rag.services import search_service

    vecs, ids, docs, groups = data
    g_hot = int(index_mod.row_group(2, 1))
    q = np.random.default_rng(5).standard_normal(DIM).astype(np.float32)
    # every row is filed under the hot group, in the mirror and the DB, except one stale row: the
    # best match, which the DB has since moved to another bot
    best = int(ids[np.argmax((vecs / np.linalg.norm(vecs, axis=1, keepdims=True)) @ q)])
    db_groups = {int(i): g_hot for i in ids}
    db_groups[best] = int(index_mod.row_group(3, 1))
    members = {pk for pk, g in db_groups.items() if g == g_hot}

    class BoundedBackend(index_mod._EngineBackend):
        asked = []

        def search(self, name, qv, n, allowed, group, doc_lt=None):
            self.asked.append(int(n))
            if not 1 <= int(n) <= index_mod.MAX_SEARCH_K:  # what gpu_service answers with a 400
                raise ValueError("k must be in [1, 1024]")
            return super().search(name, qv, n, allowed, group, doc_lt)

    svc = index_mod.IndexService(backend="engine")
    svc._be = BoundedBackend()
    name = "assistant_storage.question.embedding"
    svc._be.upsert(name, ids, vecs, docs, np.full(len(ids), g_hot, dtype=np.int32))
    monkeypatch.setattr(svc, "ensure_loaded", lambda *a: None)
    row_of = {int(i): r for r, i in enumerate(ids)}

    def meta(model, field, rows):
        pks = np.asarray([o.pk for o in rows], dtype=np.int64)
        r = np.asarray([row_of[int(p)] for p in pks], dtype=np.int64)
        return pks, docs[r], np.asarray([db_groups[int(p)] for p in pks], dtype=np.int32), vecs[r]

    monkeypatch.setattr(index_mod, "_meta_values", meta)
    qs = index_mod.with_index_filter(StubQS([]), bot=2, completed=True)
    fqs = _FilterQS(members)
    qs.filter, qs.model = fqs.filter, types.SimpleNamespace(_meta=_Meta("assistant_storage.question"), objects=fqs)
    monkeypatch.setattr(index_mod, "get_index_service", lambda: svc)
    got = asyncio.run(search_service.embedding_search_questions(q, qs, n=1000))
    assert BoundedBackend.asked == [1000, index_mod.MAX_SEARCH_K]  # the old loop asked for 2000 next
    assert len(got) == 1000
    assert all(o.pk in members for o in got)
    assert all(a.distance <= b.distance + 1e-6 for a, b in zip(got, got[1:]))
