"""``sync_to_async`` / ``async_to_sync``: asgiref's (shipped with Django) when importable, otherwise a
thread-offloading equivalent so the Django-free core (bot logic, context pipeline) runs and is
testable without Django installed."""
from __future__ import annotations

import asyncio
import functools

try:  # pragma: no cover - exercised only where Django/asgiref is installed
    from assistant.utils.sync import async_to_sync, sync_to_async  # noqa: F401
except ImportError:
    def sync_to_async(func=None, *, thread_sensitive: bool = True):
        def wrap(f):
            @functools.wraps(f)
            async def runner(*args, **kwargs):
                return await asyncio.to_thread(f, *args, **kwargs)
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
