"""Per-Instance mutual exclusion (reference bot/services/instance_service.py:15-64).

PostgreSQL: a session advisory lock keyed by the instance id (``pg_advisory_lock``), as the reference
did through django-pglocks.  Other databases (SQLite in tests, MySQL): a process-local lock per key
plus a ``SELECT ... FOR UPDATE`` row lock inside a transaction where the backend supports it -- the
same serialisation of one user's updates within a deployment."""
from __future__ import annotations

import logging
import threading
from contextlib import AbstractAsyncContextManager

from assistant.utils.sync import sync_to_async
from django.db import connection, transaction

logger = logging.getLogger(__name__)

_local_locks: dict = {}
_local_guard = threading.Lock()


def _local_lock(key: int) -> threading.RLock:
    with _local_guard:
        return _local_locks.setdefault(key, threading.RLock())


class BaseInstanceLock:
    def __init__(self, instance):
        self.instance = instance
        self.lock_key = hash(instance.id) & 0x7FFFFFFF
        self._atomic = None
        self._local = None

    def _acquire(self):
        logger.debug("acquiring instance lock %s", self.lock_key)
        if connection.vendor == "postgresql":
            with connection.cursor() as c:
                c.execute("SELECT pg_advisory_lock(%s)", [self.lock_key])
        else:
            self._local = _local_lock(self.lock_key)
            self._local.acquire()
            if connection.features.has_select_for_update:
                self._atomic = transaction.atomic()
                self._atomic.__enter__()
                type(self.instance).objects.select_for_update().filter(pk=self.instance.pk).exists()
        logger.debug("instance lock %s acquired", self.lock_key)

    def _release(self, exc_type=None, exc=None, tb=None):
        if connection.vendor == "postgresql":
            with connection.cursor() as c:
                c.execute("SELECT pg_advisory_unlock(%s)", [self.lock_key])
        else:
            if self._atomic is not None:
                self._atomic.__exit__(exc_type, exc, tb)
                self._atomic = None
            if self._local is not None:
                self._local.release()
                self._local = None
        logger.debug("instance lock %s released", self.lock_key)


class InstanceLock(BaseInstanceLock):
    def __enter__(self):
        self._acquire()
        return self

    def __exit__(self, exc_type, exc, tb):
        self._release(exc_type, exc, tb)
        return False


class InstanceLockAsync(BaseInstanceLock, AbstractAsyncContextManager):
    async def __aenter__(self):
        await sync_to_async(self._acquire, thread_sensitive=True)()
        return self

    async def __aexit__(self, exc_type, exc, tb):
        await sync_to_async(self._release, thread_sensitive=True)(exc_type, exc, tb)
        return False
