"""Per-Instance mutual exclusion (reference bot/services/instance_service.py:15-64).

Two levels, both taken in ``__enter__`` / ``__aenter__`` and dropped in reverse order:

* in-process: a non-reentrant lock per instance key.  The async form acquires it by polling from the
  coroutine, so concurrent ``answer_task`` / chat / tester coroutines for one user serialise without
  parking the thread-sensitive DB thread (a blocking acquire there would deadlock the release);
* cross-process: PostgreSQL's session advisory lock (``pg_advisory_lock``, as the reference did
  through django-pglocks), or ``SELECT ... FOR UPDATE`` inside a transaction on backends that have it.

The DB level runs through ``sync_to_async(thread_sensitive=True)``, which executes acquire and release
on the same thread and therefore the same DB connection -- a session advisory lock released from
another connection would leak (assistant/utils/sync.py).
"""
from __future__ import annotations

import asyncio
import logging
import threading
from contextlib import AbstractAsyncContextManager

from assistant.utils.sync import sync_to_async
from django.db import connection, transaction

logger = logging.getLogger(__name__)

_key_locks: dict = {}
_key_guard = threading.Lock()


def _key_lock(key: int) -> threading.Lock:
    with _key_guard:
        return _key_locks.setdefault(key, threading.Lock())


class BaseInstanceLock:
    poll_interval = 0.005

    def __init__(self, instance):
        self.instance = instance
        self.lock_key = hash(instance.id) & 0x7FFFFFFF
        self._atomic = None
        self._held = None
        self.db_thread = None  # ident of the thread that ran the DB-level acquire (tests assert on it)

    def _db_acquire(self):
        self.db_thread = threading.get_ident()
        if connection.vendor == "postgresql":
            with connection.cursor() as c:
                c.execute("SELECT pg_advisory_lock(%s)", [self.lock_key])
        elif connection.features.has_select_for_update:
            self._atomic = transaction.atomic()
            self._atomic.__enter__()
            type(self.instance).objects.select_for_update().filter(pk=self.instance.pk).exists()
        logger.debug("instance lock %s acquired", self.lock_key)

    def _db_release(self, exc_type=None, exc=None, tb=None):
        if threading.get_ident() != self.db_thread:
            logger.error("instance lock %s released on another thread than it was taken on", self.lock_key)
        if connection.vendor == "postgresql":
            with connection.cursor() as c:
                c.execute("SELECT pg_advisory_unlock(%s)", [self.lock_key])
        elif self._atomic is not None:
            self._atomic.__exit__(exc_type, exc, tb)
            self._atomic = None
        logger.debug("instance lock %s released", self.lock_key)

    def _drop_key(self):
        if self._held is not None:
            self._held.release()
            self._held = None


class InstanceLock(BaseInstanceLock):
    def __enter__(self):
        lk = _key_lock(self.lock_key)
        lk.acquire()
        self._held = lk
        try:
            self._db_acquire()
        except BaseException:
            self._drop_key()
            raise
        return self

    def __exit__(self, exc_type, exc, tb):
        try:
            self._db_release(exc_type, exc, tb)
        finally:
            self._drop_key()
        return False


class InstanceLockAsync(BaseInstanceLock, AbstractAsyncContextManager):
    async def __aenter__(self):
        lk = _key_lock(self.lock_key)
        while not lk.acquire(blocking=False):
            await asyncio.sleep(self.poll_interval)
        self._held = lk
        # The DB acquire runs on the shared thread-sensitive connection.  A cancelled coroutine
        # (timeout, client gone) must not walk away while that thread still takes the session lock:
        # the acquire is shielded, and on cancellation we wait for it to finish, release it on the
        # same thread, and only then re-raise.
        acquire = asyncio.ensure_future(sync_to_async(self._db_acquire, thread_sensitive=True)())
        try:
            await asyncio.shield(acquire)
        except asyncio.CancelledError:
            try:
                await acquire
            except BaseException:
                pass  # the acquire itself failed: nothing is held
            else:
                try:
                    await sync_to_async(self._db_release, thread_sensitive=True)(None, None, None)
                except BaseException:
                    logger.exception("instance lock %s: release after cancellation failed", self.lock_key)
            self._drop_key()
            raise
        except BaseException:
            self._drop_key()
            raise
        return self

    async def __aexit__(self, exc_type, exc, tb):
        try:
            await sync_to_async(self._db_release, thread_sensitive=True)(exc_type, exc, tb)
        finally:
            self._drop_key()
        return False
