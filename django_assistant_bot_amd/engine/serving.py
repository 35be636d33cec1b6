"""Async serving front of the engines: cross-request batching for HTTP / asyncio callers.

The reference gpu_service handlers are ``async def`` but call torch synchronously, one request at a
time per gunicorn worker, each worker holding its own full model copy.  Here one
process owns the GPU; asyncio callers submit into worker threads that batch across requests:

  * ``LLMWorker``    -- owns an ``LLMEngine`` and runs its continuous-batching step loop; every
                        awaiting caller is a sequence of the same running batch.
  * ``EmbedWorker``  -- gathers concurrent embedding requests for up to ``max_wait_s`` (or until
                        ``max_batch_tokens``) and encodes them in one packed batch.

Engines are created lazily per model name and cached for the process (``get_llm_worker`` /
``get_embed_worker``); ``engine_metrics()`` feeds gpu_service ``/metrics``.
"""
from __future__ import annotations

import asyncio
import logging
import queue
import threading
import time
from concurrent.futures import Future

logger = logging.getLogger(__name__)


class LLMWorker:
    def __init__(self, engine):
        self.engine = engine
        self._inbox: queue.Queue = queue.Queue()
        self._futures: dict[int, Future] = {}
        self._wake = threading.Event()
        self._stop = False
        self._lock = threading.Lock()
        self.requests = 0
        self.faults = 0
        self.healthy = True  # False after a sticky device error: /health reports 503 for a restart
        self.last_error = ""
        self._thread = threading.Thread(target=self._run, name="dab-llm-worker", daemon=True)
        self._thread.start()

    def submit(self, prompt_ids, params) -> Future:
        fut: Future = Future()
        self._inbox.put((list(prompt_ids), params, fut))
        self._wake.set()
        return fut

    async def generate(self, prompt_ids, params):
        fut = self.submit(prompt_ids, params)
        try:
            return await asyncio.wrap_future(fut)
        except asyncio.CancelledError:  # caller gone (client disconnect / timeout): free its slot
            self.cancel(fut)
            raise

    def cancel(self, fut: Future) -> None:
        self._inbox.put(("__cancel__", None, fut))
        self._wake.set()

    def _drain(self):
        while True:
            try:
                ids, params, fut = self._inbox.get_nowait()
            except queue.Empty:
                return
            if ids == "__cancel__":
                for rid, f in list(self._futures.items()):
                    if f is fut:
                        self.engine.abort(rid, "cancelled")
                        self.engine.pop_output(rid)
                        del self._futures[rid]
                continue
            try:
                rid = self.engine.add_request(ids, params)
                self._futures[rid] = fut
                self.requests += 1
            except Exception as exc:  # invalid request: fail only this caller
                fut.set_exception(exc)

    def _run(self):
        while not self._stop:
            self._drain()
            if not self.engine.has_unfinished():
                self._wake.wait(0.05)
                self._wake.clear()
                continue
            try:
                finished = self.engine.step()
            except Exception as exc:  # engine fault: fail every in-flight request, keep serving
                logger.exception("engine step failed")
                self.faults += 1
                self.last_error = f"{type(exc).__name__}: {exc}"
                if _sticky_device_error(exc):
                    # a HIP fault poisons the context: stop taking work, let the supervisor restart
                    self.healthy = False
                for fut in self._futures.values():
                    if not fut.done():
                        fut.set_exception(exc)
                self._futures.clear()
                self.engine.fail_all()
                continue
            for rid in finished:
                fut = self._futures.pop(rid, None)
                out = self.engine.pop_output(rid)
                if fut is None or fut.done():
                    continue
                if out is not None and out.finish_reason.startswith("error:"):  # refused by a replica
                    fut.set_exception(RuntimeError(f"request refused by the engine ({out.finish_reason})"))
                else:
                    fut.set_result(out)

    def stop(self):
        self._stop = True
        self._wake.set()

    def join(self, timeout: float | None = None) -> None:
        self._thread.join(timeout)


def _sticky_device_error(exc: BaseException) -> bool:
    """HIP errors that leave the device context unusable (memory faults, illegal instructions,
    ECC, hardware exceptions), and a broken TP group (a peer missed a one-shot all-reduce: every
    later reduction on this rank is poisoned); after one the process must be restarted."""
    from ..parallel.custom_allreduce import CustomAllReduceError

    if isinstance(exc, CustomAllReduceError):
        return True
    msg = str(exc).lower()
    return any(k in msg for k in ("illegal address", "illegal memory access", "memory access fault", "hiperrorillegal", "ecc error",
                                  "hardware exception", "device-side assert", "unspecified launch failure",
                                  "hiperrorlaunchfailure", "device lost"))


class EmbedWorker:
    def __init__(self, engine, max_wait_s: float = 0.002, max_batch_texts: int = 4096):
        self.engine = engine
        self.max_wait_s = max_wait_s
        self.max_batch_texts = max_batch_texts
        self._inbox: queue.Queue = queue.Queue()
        self._concurrent = False
        self.requests = 0
        self._thread = threading.Thread(target=self._run, name="dab-embed-worker", daemon=True)
        self._thread.start()

    def submit(self, texts, normalize=None) -> Future:
        fut: Future = Future()
        self._inbox.put((list(texts), normalize, fut))
        return fut

    async def embeddings(self, texts, normalize=None):
        return await asyncio.wrap_future(self.submit(texts, normalize))

    def _run(self):
        while True:
            first = self._inbox.get()
            batch = [first]
            n = len(first[0])
            # wait for company only when callers have recently been concurrent; a lone sequential
            # client gets no added latency (requests already queued are always taken)
            wait = self.max_wait_s if self._concurrent else 0.0
            deadline = time.perf_counter() + wait
            while n < self.max_batch_texts:
                left = deadline - time.perf_counter()
                try:
                    item = self._inbox.get(timeout=left) if left > 0 else self._inbox.get_nowait()
                except queue.Empty:
                    break
                batch.append(item)
                n += len(item[0])
            self._concurrent = len(batch) > 1 or not self._inbox.empty()
            groups: dict = {}
            for texts, norm, fut in batch:
                groups.setdefault(norm, []).append((texts, fut))
            for norm, items in groups.items():
                flat = [t for texts, _ in items for t in texts]
                try:
                    vecs = self.engine.embed(flat, normalize=norm).float().cpu().tolist() if flat else []
                except Exception as exc:
                    for _, fut in items:
                        fut.set_exception(exc)
                    continue
                o = 0
                for texts, fut in items:
                    fut.set_result(vecs[o:o + len(texts)])
                    o += len(texts)
                self.requests += len(items)


_llm: dict = {}
_emb: dict = {}
_lock = threading.Lock()


def setting(name: str, default):
    """Engine setting (SURVEY.md 5.6 keys) from the app settings when available, else the env."""
    try:
        from assistant.conf import settings

        v = settings.get(name, default)
    except ImportError:
        import os

        v = os.environ.get(name, default)
    if v is None or default is None:
        return v
    return type(default)(v)


def engine_device():
    """``GPU_SERVICE_DEVICE`` (e.g. ``cpu`` for the plumbing-only config) overrides the default."""
    import os

    import torch

    forced = os.environ.get("GPU_SERVICE_DEVICE")
    if forced:
        return forced
    return "cuda" if torch.cuda.is_available() else "cpu"


def get_llm_worker(model: str, **engine_kwargs) -> LLMWorker:
    key = model.lower()
    with _lock:
        w = _llm.get(key)
        if w is None:
            from .llm_engine import LLMEngine

            engine_kwargs.setdefault("device", engine_device())
            engine_kwargs.setdefault("max_batch", 64 if engine_kwargs["device"] == "cuda" else 4)
            engine_kwargs.setdefault("block_size", setting("KV_BLOCK_SIZE", 64))
            engine_kwargs.setdefault("max_prefill_tokens", setting("MAX_BATCH_TOKENS", 65536))
            if engine_kwargs["device"] == "cpu":
                engine_kwargs.setdefault("max_model_len", 2048)
            w = _llm[key] = LLMWorker(LLMEngine(model, **engine_kwargs))
        return w


def get_embed_worker(model: str, **engine_kwargs) -> EmbedWorker:
    key = model.lower()
    with _lock:
        w = _emb.get(key)
        if w is None:
            from .embedding_engine import EmbeddingEngine

            engine_kwargs.setdefault("device", engine_device())
            w = _emb[key] = EmbedWorker(EmbeddingEngine(model, **engine_kwargs))
        return w


_node = None  # the gpu_service node (parallel.node.Node) when running in node mode


def health() -> dict:
    """Worker health for gpu_service /health (unhealthy after a sticky device fault, or when the
    node's process group broke)."""
    bad = {k: w.last_error for k, w in _llm.items() if not w.healthy}
    if _node is not None and not _node.healthy:
        bad["node"] = _node.last_error
    return {"healthy": not bad, "unhealthy_workers": bad}


def engine_metrics() -> dict:
    import torch

    m = {"embedders": {}, "providers": {}}
    for k, w in _emb.items():
        m["embedders"][k] = {"requests": w.requests, **w.engine.stats, "queue_depth": w._inbox.qsize()}
    for k, w in _llm.items():
        e = w.engine
        m["providers"][k] = {"requests": w.requests, "faults": w.faults, "healthy": int(w.healthy), **e.stats, "running": len(e.running), "waiting": len(e.waiting),
                             "kv_free_blocks": e.blocks.num_free_blocks(), "kv_total_blocks": e.blocks.num_blocks(),
                             "prefix_hit_tokens": e.blocks.prefix_hits()}
    if torch.cuda.is_available():
        free, total = torch.cuda.mem_get_info()
        m["hbm"] = {"free_gb": round(free / 2 ** 30, 2), "total_gb": round(total / 2 ** 30, 2)}
    return m
