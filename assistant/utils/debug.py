"""``debug_info`` timing context manager (reference utils/debug.py:5-30)."""
from __future__ import annotations

import time


class TimeDebugger:
    def __init__(self, debug_info: dict, key: str | None = None):
        if key:
            self.info = debug_info.setdefault(key, {})
        else:
            self.info = debug_info
        self._t0: float | None = None
        self._took: float | None = None

    def __enter__(self):
        self._t0 = time.perf_counter()
        return self

    def __exit__(self, exc_type, exc, tb):
        self._took = time.perf_counter() - self._t0
        self.info["took"] = self._took
        return False

    @property
    def execution_time(self) -> float:
        if self._took is not None:
            return self._took
        return time.perf_counter() - (self._t0 or time.perf_counter())
