"""gpu_service HTTP API on CPU with the tiny engine presets (FastAPI TestClient): embeddings, dialog,
vector-index upsert/search/delete, health and Prometheus metrics; error codes of the reference
(400 unknown model)."""
import pytest

fastapi = pytest.importorskip("fastapi")
from fastapi.testclient import TestClient  # noqa: E402

from gpu_service import main as svc  # noqa: E402


@pytest.fixture(scope="module")
def client():
    svc.embedders.clear()
    svc.providers.clear()
    svc.indexes.clear()
    svc.load_models(["tiny-bert"], ["tiny-llama"])
    app = svc.FastAPI()  # no lifespan: models loaded above
    for r in svc.app.routes:
        app.router.routes.append(r)
    return TestClient(app)


def test_embeddings(client):
    r = client.post("/embeddings/", json={"model": "TINY-BERT", "texts": ["hello world", "привет мир"]})
    assert r.status_code == 200
    e = r.json()["embeddings"]
    assert len(e) == 2 and len(e[0]) == 128
    assert client.post("/embeddings/", json={"model": "nope", "texts": ["x"]}).status_code == 400


def test_dialog(client):
    r = client.post("/dialog/", json={"model": "tiny-llama", "messages": [{"role": "user", "content": "hi"}],
                                      "max_tokens": 5})
    assert r.status_code == 200
    resp = r.json()["response"]
    assert resp["usage"]["completion_tokens"] <= 5 and isinstance(resp["result"], str)
    assert resp["length_limited"] in (True, False)
    assert client.post("/dialog/", json={"model": "x", "messages": []}).status_code == 400


def test_dialog_json_schema(client):
    """/dialog/ with a JSON Schema (an extension of the reference schema): the answer is an object;
    a schema the constrained decoder cannot compile is a 400, not a 500."""
    msg = [{"role": "user", "content": "json please"}]
    schema = {"type": "object", "properties": {"question": {"type": ["integer", "null"]}}}
    r = client.post("/dialog/", json={"model": "tiny-llama", "messages": msg, "max_tokens": 16,
                                      "json_format": True, "json_schema": schema})
    assert r.status_code == 200 and isinstance(r.json()["response"]["result"], dict)
    bad = client.post("/dialog/", json={"model": "tiny-llama", "messages": msg, "json_schema": {"type": "string"}})
    assert bad.status_code == 400


def test_index_roundtrip(client):
    vecs = [[1.0, 0.0, 0.0, 0.0], [0.0, 1.0, 0.0, 0.0], [0.7, 0.7, 0.0, 0.0]]
    r = client.post("/index/q/upsert", json={"ids": [10, 11, 12], "vectors": vecs, "doc_ids": [1, 2, 3]})
    assert r.json() == {"count": 3}
    r = client.post("/index/q/search", json={"queries": [[1.0, 0.1, 0.0, 0.0]], "k": 2}).json()
    assert r["ids"][0] == [10, 12] and r["doc_ids"][0] == [1, 3]
    assert r["distances"][0][0] < r["distances"][0][1]
    r = client.post("/index/q/search", json={"queries": [[1.0, 0.1, 0.0, 0.0]], "k": 3, "allowed": [[11, 12]]}).json()
    assert r["ids"][0] == [12, 11]
    assert client.post("/index/q/delete", json={"ids": [12]}).json() == {"removed": 1}
    r = client.post("/index/q/search", json={"queries": [[1.0, 0.1, 0.0, 0.0]], "k": 3}).json()
    assert r["ids"][0] == [10, 11]
    assert client.post("/index/none/search", json={"queries": [[1, 0, 0, 0]], "k": 3}).json()["ids"] == [[]]


def test_index_ingest_single_process(client):
    texts = ["alpha beta", "gamma delta", "epsilon zeta"]
    r = client.post("/index/docs/ingest", json={"model": "TINY-BERT", "ids": [5, 6, 7], "texts": texts,
                                                "doc_ids": [1, 1, 2], "return_vectors": True}).json()
    assert r["count"] == 3 and len(r["embeddings"]) == 3
    q = client.post("/embeddings/", json={"model": "tiny-bert", "texts": [texts[1]]}).json()["embeddings"]
    hit = client.post("/index/docs/search", json={"queries": q, "k": 1}).json()
    assert hit["ids"] == [[6]] and hit["doc_ids"] == [[1]]
    assert client.post("/index/docs/ingest", json={"model": "x", "ids": [1], "texts": ["a"]}).status_code == 400
    assert client.post("/index/docs/ingest", json={"model": "tiny-bert", "ids": [1], "texts": []}).status_code == 400


def test_health_and_metrics(client):
    h = client.get("/health").json()
    assert h["status"] == "ok" and "tiny-bert" in h["embedders"] and "tiny-llama" in h["providers"]
    m = client.get("/metrics").text
    assert 'dab_embedder_requests{model="tiny-bert"}' in m
    assert 'dab_provider_requests{model="tiny-llama"}' in m


def test_gunicorn_device_mapping_survives_respawn(monkeypatch):
    """A respawned worker takes the GPU its predecessor left (reference gunicorn_conf.py ran every
    worker on one device; worker.age-based mapping drifted after restarts)."""
    from types import SimpleNamespace

    from gpu_service import gunicorn_conf as gc

    monkeypatch.setattr(gc, "devices", 4)
    live = {}
    for pid in range(4):
        w = SimpleNamespace()
        gc.pre_fork(SimpleNamespace(WORKERS=live), w)
        live[pid] = w
    assert sorted(w.dab_device for w in live.values()) == [0, 1, 2, 3]
    dead = live.pop(2)
    w = SimpleNamespace()
    gc.pre_fork(SimpleNamespace(WORKERS=live), w)
    assert w.dab_device == dead.dab_device
    assert gc.pick_device([SimpleNamespace(dab_device=d) for d in (0, 1, 2, 3)], 4) == 0  # oversubscribed
    assert gc.pick_device([SimpleNamespace(dab_device=d) for d in (0, 2)], 4) == 1


def test_index_refused_with_independent_workers(client, monkeypatch):
    monkeypatch.setenv("GPU_SERVICE_WORKERS", "2")
    r = client.post("/index/q/search", json={"queries": [[1.0, 0.0, 0.0, 0.0]], "k": 1})
    assert r.status_code == 409
