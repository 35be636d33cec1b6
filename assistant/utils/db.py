"""Temporarily strip Django model signal receivers (reference utils/db.py:8-43); receivers are
always restored, also when the body raises."""
from __future__ import annotations

from contextlib import contextmanager


@contextmanager
def disable_signals(model=None, signals=None):
    from django.db.models.signals import (m2m_changed, post_delete, post_init, post_save, pre_delete, pre_init,
                                          pre_save)

    if signals is None:
        signals = [pre_save, post_save, pre_delete, post_delete, m2m_changed, pre_init, post_init]
    saved = {}
    for sig in signals:
        with sig.lock:
            saved[sig] = list(sig.receivers)
            if model is None:
                sig.receivers = []
            else:
                sig.receivers = [r for r in sig.receivers if r[0][1] != id(model)]
            sig.sender_receivers_cache.clear()
    try:
        yield
    finally:
        for sig, receivers in saved.items():
            with sig.lock:
                sig.receivers = receivers
                sig.sender_receivers_cache.clear()
