"""Minimum-interval async throttle (reference utils/throttle.py:9-30), safe under concurrent callers."""
from __future__ import annotations

import asyncio
import time


class Throttle:
    def __init__(self, time_period: float):
        self.time_period = float(time_period)
        self.last_call = 0.0
        self._lock: asyncio.Lock | None = None

    async def __call__(self) -> None:
        if self._lock is None:
            self._lock = asyncio.Lock()
        async with self._lock:
            wait = self.time_period - (time.monotonic() - self.last_call)
            if wait > 0:
                await asyncio.sleep(wait)
            self.last_call = time.monotonic()
