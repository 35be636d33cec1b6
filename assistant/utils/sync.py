"""``sync_to_async`` / ``async_to_sync``: asgiref's (shipped with Django) when importable, otherwise an
equivalent with the same thread semantics, so the Django-free core (bot logic, context pipeline) runs
and is testable without Django installed.

The fallback keeps asgiref's contract that matters for correctness: every ``thread_sensitive=True``
call runs on ONE dedicated thread (asgiref: the main thread / a single shared executor).  Code that
binds state to a thread -- a DB connection, a session advisory lock taken in ``__aenter__`` and
released in ``__aexit__`` (bot/services/instance_service.py) -- therefore always sees the same thread.
``thread_sensitive=False`` calls go to the default thread pool.
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import functools
import threading

try:  # pragma: no cover - exercised only where Django/asgiref is installed
    from asgiref.sync import async_to_sync, sync_to_async  # noqa: F401

    HAVE_ASGIREF = True
except ImportError:
    HAVE_ASGIREF = False

    _sensitive_lock = threading.Lock()
    _sensitive_executor: concurrent.futures.ThreadPoolExecutor | None = None

    def _executor() -> concurrent.futures.ThreadPoolExecutor:
        global _sensitive_executor
        with _sensitive_lock:
            if _sensitive_executor is None:
                _sensitive_executor = concurrent.futures.ThreadPoolExecutor(
                    max_workers=1, thread_name_prefix="thread-sensitive")
            return _sensitive_executor

    def sensitive_thread_ident() -> int:
        """Ident of the single thread that runs thread-sensitive calls (for tests / assertions)."""
        return _executor().submit(threading.get_ident).result()

    def sync_to_async(func=None, *, thread_sensitive: bool = True):
        def wrap(f):
            @functools.wraps(f)
            async def runner(*args, **kwargs):
                call = functools.partial(f, *args, **kwargs)
                if thread_sensitive:
                    if threading.current_thread().name.startswith("thread-sensitive"):
                        return call()  # already on the sensitive thread (nested call)
                    return await asyncio.wrap_future(_executor().submit(call))
                return await asyncio.to_thread(call)
            return runner
        return wrap(func) if func is not None else wrap

    def async_to_sync(coro_fn):
        @functools.wraps(coro_fn)
        def runner(*args, **kwargs):
            try:
                asyncio.get_running_loop()
            except RuntimeError:
                return asyncio.run(coro_fn(*args, **kwargs))
            raise RuntimeError("async_to_sync called from a running event loop")
        return runner
