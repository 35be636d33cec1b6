"""Tracing: roctx ranges and HIP-event GPU phase timings.

The reference's only instrumentation is the per-request ``debug_info`` dict of host wall times
(reference utils/debug.py:5-30, ai/providers/base.py:48-70).  That is kept by the app layer; the
engine adds two things a host timer cannot see:

* ``range(name)`` -- a roctx range around an engine phase (``llm.prefill``, ``llm.decode``,
  ``embed``, ``index.search`` ...), so ``rocprofv3 --marker-trace --kernel-trace`` attributes every
  kernel to the phase that launched it.  Off unless ``DAB_ROCTX=1`` (or ``set_roctx(True)``); the
  native side resolves the roctx library lazily and is a no-op without it.
* ``GpuTimer`` -- named GPU spans from HIP event pairs recorded on the current stream.  ``collect``
  is meant to be called where the host synchronises anyway (after a decode step's token copy, after
  the search results come back), so timing adds no stalls.  A span is the device-side time from the
  start event to the end event, idle gaps included.
"""
from __future__ import annotations

import contextlib
import os

import torch

_roctx = os.environ.get("DAB_ROCTX", "0") == "1"


def set_roctx(flag: bool) -> None:
    global _roctx
    _roctx = bool(flag)


def roctx_enabled() -> bool:
    return _roctx


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    if not _roctx:
        yield
        return
    from ..ops._lib import native

    n = native()
    n.roctx_push(name)
    try:
        yield
    finally:
        n.roctx_pop()


def mark(name: str) -> None:
    if _roctx:
        from ..ops._lib import native

        native().roctx_mark(name)


class GpuTimer:
    """Accumulates named GPU spans (ms).  Disabled (every call a no-op) on CPU or when
    ``enabled=False``; ``DAB_GPU_TIMING=0`` turns engine timers off globally."""

    def __init__(self, enabled: bool = True, device=None):
        on = enabled and os.environ.get("DAB_GPU_TIMING", "1") != "0"
        self.enabled = bool(on and torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda"))
        self._pending: list = []
        self._free: list = []
        self.totals: dict[str, float] = {}
        self.counts: dict[str, int] = {}

    def _event(self):
        return self._free.pop() if self._free else torch.cuda.Event(enable_timing=True)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            with range(name):
                yield
            return
        start, end = self._event(), self._event()
        start.record()
        try:
            with range(name):
                yield
        finally:
            end.record()
            self._pending.append((name, start, end))

    def collect(self, block: bool = True) -> dict[str, float]:
        """Resolve the recorded spans -> {name: ms} since the last collect.  ``block=False`` takes
        only the spans whose end event has already completed and leaves the rest pending."""
        out: dict[str, float] = {}
        keep = []
        for name, start, end in self._pending:
            if not block and not end.query():
                keep.append((name, start, end))
                continue
            end.synchronize()
            ms = start.elapsed_time(end)
            out[name] = out.get(name, 0.0) + ms
            self.totals[name] = self.totals.get(name, 0.0) + ms
            self.counts[name] = self.counts.get(name, 0) + 1
            self._free += (start, end)
        self._pending = keep
        return out

    def reset(self) -> None:
        self.collect()
        self.totals.clear()
        self.counts.clear()
