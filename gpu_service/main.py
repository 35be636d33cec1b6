"""gpu_service: embeddings, dialog, vector index and metrics over HTTP (reference gpu_service/main.py).

Endpoints (request/response shapes of the reference where it had them):
  POST /embeddings/             {model, texts}                         -> {embeddings: [[float]]}
  POST /dialog/                 {model, messages, max_tokens, json_format[, json_schema]} -> {response: AIResponse}
  POST /index/{name}/upsert     {ids, vectors, doc_ids?, groups?}      -> {count}
  POST /index/{name}/delete     {ids}                                  -> {removed}
  POST /index/{name}/search     {queries, k, groups?, allowed?}        -> {ids, distances, doc_ids}
  POST /index/{name}/ingest     {model, ids, texts, doc_ids?, groups?, return_vectors?}
                                -> {count[, embeddings]}  (embed + upsert; rank-local in node mode)
  GET  /health                  loaded models, device
  GET  /metrics                 Prometheus text (engine counters, queue depths, HBM use)

Requests from all concurrent callers share the engine's batches (EmbedWorker / LLMWorker).  Two
deployments:

* one process per GPU under gunicorn (``gunicorn_conf.py``): independent replicas for /embeddings/
  and /dialog/; /index/* needs a single worker (409 otherwise -- replicas would hold different indexes);
* node mode (``python -m torch.distributed.run --nproc-per-node N -m gpu_service.node_main``): one
  process group over the node's GPUs -- sharded index, DP embeddings, TP / replicated generators
  (``django_assistant_bot_amd.parallel.node``).  The handlers below are the same; ``index_backend``
  and the engine workers are swapped for the node facades.

Model names are case-insensitive; unknown model -> 400; engine errors -> 500.
"""
from __future__ import annotations

import logging
import os
import sys
import threading
from contextlib import asynccontextmanager
from dataclasses import asdict
from typing import Dict, List, Optional

from fastapi import FastAPI, HTTPException
from fastapi.responses import PlainTextResponse
from starlette.concurrency import run_in_threadpool
from pydantic import BaseModel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from django_assistant_bot_amd.engine.json_schema import SchemaError  # noqa: E402

logging.basicConfig(level=os.environ.get("GPU_SERVICE_LOG_LEVEL", "INFO"),
                    format="%(asctime)s - %(name)s - %(levelname)s - %(message)s")
logger = logging.getLogger("gpu_service")


class EmbeddingRequest(BaseModel):
    model: str
    texts: List[str]


class Message(BaseModel):
    role: str
    content: str


class DialogRequest(BaseModel):
    model: str
    messages: List[Message]
    max_tokens: int = 1024
    json_format: bool = False
    json_schema: Optional[dict] = None  # constrained decoding to a JSON Schema (engine/json_schema.py)


class UpsertRequest(BaseModel):
    ids: List[int]
    vectors: List[List[float]]
    doc_ids: Optional[List[int]] = None
    groups: Optional[List[int]] = None


class IngestRequest(BaseModel):
    model: str
    ids: List[int]
    texts: List[str]
    doc_ids: Optional[List[int]] = None
    groups: Optional[List[int]] = None
    return_vectors: bool = False


class DeleteRequest(BaseModel):
    ids: List[int]


class SearchRequest(BaseModel):
    queries: List[List[float]]
    k: int = 10
    groups: Optional[List[int]] = None
    allowed: Optional[List[List[int]]] = None
    doc_lt: Optional[List[int]] = None


embedders: Dict[str, object] = {}
providers: Dict[str, object] = {}
indexes: Dict[str, object] = {}


def load_models(embedder_names, provider_names):
    from assistant.ai.embedders.transformers import TransformersEmbedder
    from assistant.ai.providers.transformers import TransformersProvider

    for name in embedder_names:
        try:
            embedders[name.lower()] = TransformersEmbedder(name)
        except Exception:
            logger.exception("failed to load embedder %s", name)
    for name in provider_names:
        try:
            providers[name.lower()] = TransformersProvider(name)
        except Exception:
            logger.exception("failed to load provider %s", name)
    logger.info("serving embedders=%s providers=%s", sorted(embedders), sorted(providers))


@asynccontextmanager
async def lifespan(app: FastAPI):
    from gpu_service.models import embedder_models, provider_models

    load_models(embedder_models, provider_models)
    yield


app = FastAPI(title="gpu_service", lifespan=lifespan)


@app.post("/embeddings/")
async def get_embeddings(request: EmbeddingRequest):
    embedder = embedders.get(request.model.lower())
    if embedder is None:
        raise HTTPException(status_code=400, detail="Model is not supported")
    try:
        return {"embeddings": await embedder.embeddings(request.texts)}
    except Exception as e:
        logger.exception("embeddings failed")
        raise HTTPException(status_code=500, detail=str(e))


@app.post("/dialog/")
async def get_response(request: DialogRequest):
    provider = providers.get(request.model.lower())
    if provider is None:
        raise HTTPException(status_code=400, detail="Model is not supported")
    try:
        kw = {"json_schema": request.json_schema} if request.json_schema is not None else {}
        resp = await provider.get_response([{"role": m.role, "content": m.content} for m in request.messages],
                                           max_tokens=request.max_tokens, json_format=request.json_format, **kw)
        return {"response": asdict(resp)}
    except SchemaError as e:  # a JSON Schema the constrained decoder cannot compile: the client's fault
        raise HTTPException(status_code=400, detail=str(e))
    except Exception as e:
        logger.exception("dialog failed")
        raise HTTPException(status_code=500, detail=str(e))


class LocalIndexes:
    """Single-process ``/index/*`` backend: one ``VectorIndex`` per name on this process's GPU.
    (Node mode replaces it with ``NodeIndexes``: one index sharded over the node's GPUs.)"""

    def __init__(self, store: Dict[str, object]):
        self.indexes = store
        self._lock = threading.Lock()

    def dim(self, name: str):
        idx = self.indexes.get(name)
        return None if idx is None else idx.dim

    def upsert(self, name, ids, vectors, doc_ids=None, groups=None) -> int:
        for what, v in (("doc_ids", doc_ids), ("groups", groups)):
            if v is not None and len(v) != len(ids):
                raise ValueError(f"{what} must hold one entry per id")
        if groups is not None and any(g < 0 for g in groups):
            raise ValueError("groups must be >= 0")
        with self._lock:
            idx = self.indexes.get(name)
            if idx is None:
                import torch

                from django_assistant_bot_amd.engine.serving import engine_device, setting
                from django_assistant_bot_amd.engine.vector_index import VectorIndex

                dtype = getattr(torch, str(setting("INDEX_DTYPE", "bfloat16")))
                idx = self.indexes[name] = VectorIndex(len(vectors[0]), device=engine_device(), dtype=dtype)
            idx.add(ids, vectors, doc_ids=doc_ids, groups=groups)
            return len(idx)

    def delete(self, name, ids) -> int:
        with self._lock:
            idx = self.indexes.get(name)
            return 0 if idx is None else idx.remove(ids)

    def size(self, name) -> int:
        idx = self.indexes.get(name)
        return 0 if idx is None else len(idx)

    def search(self, name, queries, k, groups=None, allowed=None, doc_lt=None):
        nq = len(queries)
        if not 1 <= int(k) <= 1024:
            raise ValueError("k must be in [1, 1024]")
        for what, v in (("groups", groups), ("allowed", allowed), ("doc_lt", doc_lt)):
            if v is not None and len(v) != nq:
                raise ValueError(f"{what} must hold one entry per query")
        with self._lock:
            idx = self.indexes.get(name)
            if idx is None or len(idx) == 0:
                return None
            return idx.search(queries, k, q_groups=groups, allowed=allowed, doc_lt=doc_lt)

    def sizes(self) -> dict:
        return {k: len(v) for k, v in self.indexes.items()}


index_backend = LocalIndexes(indexes)


def _workers_share_nothing() -> bool:
    """gunicorn with several workers = independent replicas: an index would differ per worker."""
    return int(os.environ.get("GPU_SERVICE_WORKERS", "1")) > 1 and isinstance(index_backend, LocalIndexes)


def _index_guard():
    if _workers_share_nothing():
        raise HTTPException(status_code=409, detail="/index/* needs one index: run gpu_service.node_main "
                                                    "(one process group over the node's GPUs) or one worker")


async def _call_index(fn, *args):
    """Index backends raise ValueError for a malformed payload (lengths, dims, k, negative groups):
    that is the caller's error (400), and in node mode it is raised before anything reaches the
    other ranks, so the group stays healthy."""
    try:
        return await run_in_threadpool(fn, *args)
    except ValueError as e:
        raise HTTPException(status_code=400, detail=str(e))


@app.post("/index/{name}/upsert")
async def index_upsert(name: str, request: UpsertRequest):
    _index_guard()
    if len(request.ids) != len(request.vectors):
        raise HTTPException(status_code=400, detail="ids and vectors differ in length")
    if not request.ids:
        return {"count": index_backend.size(name)}
    dim = index_backend.dim(name)
    if dim is not None and len(request.vectors[0]) != dim:
        raise HTTPException(status_code=400, detail=f"index {name} has dim {dim}")
    n = await _call_index(index_backend.upsert, name, request.ids, request.vectors, request.doc_ids, request.groups)
    return {"count": n}


@app.post("/index/{name}/ingest")
async def index_ingest(name: str, request: IngestRequest):
    """Document ingest in one call: embed the texts and write them into the index.  Node mode runs
    it where the rows live (each text goes to the rank owning its shard, which embeds it and writes
    its own shard from HBM: no vector crosses a link); one process embeds then upserts."""
    _index_guard()
    if len(request.ids) != len(request.texts):
        raise HTTPException(status_code=400, detail="ids and texts differ in length")
    if hasattr(index_backend, "ingest"):
        out = await _call_index(index_backend.ingest, name, request.model, request.ids, request.texts,
                                request.doc_ids, request.groups, None, request.return_vectors)
        if request.return_vectors:
            return {"count": out[0], "embeddings": out[1].tolist()}
        return {"count": out}
    embedder = embedders.get(request.model.lower())
    if embedder is None:
        raise HTTPException(status_code=400, detail="Model is not supported")
    if not request.ids:
        return {"count": index_backend.size(name), **({"embeddings": []} if request.return_vectors else {})}
    vecs = await embedder.embeddings(request.texts)
    dim = index_backend.dim(name)
    if dim is not None and len(vecs[0]) != dim:
        raise HTTPException(status_code=400, detail=f"index {name} has dim {dim}")
    n = await _call_index(index_backend.upsert, name, request.ids, vecs, request.doc_ids, request.groups)
    return {"count": n, **({"embeddings": vecs} if request.return_vectors else {})}


@app.post("/index/{name}/delete")
async def index_delete(name: str, request: DeleteRequest):
    _index_guard()
    return {"removed": await _call_index(index_backend.delete, name, request.ids)}


@app.post("/index/{name}/search")
async def index_search(name: str, request: SearchRequest):
    _index_guard()
    nq = len(request.queries)
    got = None
    if nq:
        got = await _call_index(index_backend.search, name, request.queries, request.k, request.groups,
                                request.allowed, request.doc_lt)
    if got is None:
        return {"ids": [[] for _ in range(nq)], "distances": [[] for _ in range(nq)],
                "doc_ids": [[] for _ in range(nq)]}
    sims, ids, docs = got
    out_ids, out_d, out_docs = [], [], []
    for s, i, d in zip(sims.tolist(), ids.tolist(), docs.tolist()):
        keep = [j for j, x in enumerate(i) if x >= 0]
        out_ids.append([i[j] for j in keep])
        out_d.append([1.0 - s[j] for j in keep])
        out_docs.append([d[j] for j in keep])
    return {"ids": out_ids, "distances": out_d, "doc_ids": out_docs}


@app.get("/health")
async def health():
    """200 when serving; 503 after a sticky device fault in an engine worker (the supervisor /
    gunicorn restarts the process)."""
    from fastapi.responses import JSONResponse

    from django_assistant_bot_amd.engine.serving import engine_device, health as engine_health

    h = engine_health()
    body = {"status": "ok" if h["healthy"] else "unhealthy", "device": str(engine_device()),
            "embedders": sorted(embedders), "providers": sorted(providers),
            "indexes": index_backend.sizes(), **({} if h["healthy"] else h)}
    return JSONResponse(body, status_code=200 if h["healthy"] else 503)


def _flatten(prefix: str, obj, out: list, labels: str = ""):
    if isinstance(obj, dict):
        for k, v in obj.items():
            if isinstance(v, dict) and k in ("embedders", "providers"):
                for model, stats in v.items():
                    _flatten(f"{prefix}_{k[:-1]}", stats, out, f'model="{model}"')
            else:
                _flatten(f"{prefix}_{k}", v, out, labels)
    elif isinstance(obj, (int, float)) and not isinstance(obj, bool):
        out.append(f"{prefix}{{{labels}}} {float(obj)}" if labels else f"{prefix} {float(obj)}")


@app.get("/metrics", response_class=PlainTextResponse)
async def metrics():
    from django_assistant_bot_amd.engine.serving import engine_metrics

    lines: list = []
    _flatten("dab", engine_metrics(), lines)
    lines += [f'dab_index_rows{{index="{k}"}} {float(v)}' for k, v in index_backend.sizes().items()]
    return "\n".join(lines) + "\n"
