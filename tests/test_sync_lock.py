"""The sync_to_async shim and the per-instance lock (reference bot/services/instance_service.py:52-64).

Django is not installed here, so ``django.db`` is replaced by a stub that records on which thread the
DB-level acquire / release run; the lock logic itself is the production module.
"""
import asyncio
import importlib
import sys
import threading
import types

import pytest

from assistant.utils import sync as sync_mod


@pytest.fixture()
def instance_service(monkeypatch):
    calls = []

    class Cursor:
        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

        def execute(self, sql, args):
            calls.append((sql.split("(")[0], threading.get_ident()))

    conn = types.SimpleNamespace(vendor="postgresql", cursor=lambda: Cursor(),
                                 features=types.SimpleNamespace(has_select_for_update=True))
    db = types.ModuleType("django.db")
    db.connection = conn
    db.transaction = types.SimpleNamespace(atomic=lambda: None)
    django = types.ModuleType("django")
    django.db = db
    monkeypatch.setitem(sys.modules, "django", django)
    monkeypatch.setitem(sys.modules, "django.db", db)
    sys.modules.pop("assistant.bot.services.instance_service", None)
    mod = importlib.import_module("assistant.bot.services.instance_service")
    yield mod, calls
    sys.modules.pop("assistant.bot.services.instance_service", None)


def test_shim_is_not_a_self_import():
    src = open(sync_mod.__file__).read()
    assert "from assistant.utils.sync import" not in src
    assert "from asgiref.sync import" in src


def test_thread_sensitive_calls_share_one_thread():
    if sync_mod.HAVE_ASGIREF:
        pytest.skip("asgiref installed: its own semantics apply")

    async def main():
        idents = await asyncio.gather(*[sync_mod.sync_to_async(threading.get_ident)() for _ in range(16)])
        return set(idents)

    idents = asyncio.run(main())
    assert idents == {sync_mod.sensitive_thread_ident()}
    assert threading.get_ident() not in idents


def test_async_lock_acquires_and_releases_on_one_thread(instance_service):
    mod, calls = instance_service

    async def main():
        async with mod.InstanceLockAsync(types.SimpleNamespace(id=42)):
            await asyncio.sleep(0)
            # unrelated thread-sensitive work between acquire and release
            await asyncio.gather(*[sync_mod.sync_to_async(lambda: None)() for _ in range(8)])

    asyncio.run(main())
    assert [c[0] for c in calls] == ["SELECT pg_advisory_lock", "SELECT pg_advisory_unlock"]
    assert calls[0][1] == calls[1][1], "advisory lock released on a different thread / connection"


def test_concurrent_holders_of_one_instance_serialise(instance_service):
    mod, calls = instance_service
    inst = types.SimpleNamespace(id=7)
    events = []

    async def answer_update(tag):
        async with mod.InstanceLockAsync(inst):
            events.append(("in", tag))
            await asyncio.sleep(0.02)
            events.append(("out", tag))

    async def main():
        await asyncio.gather(*[answer_update(i) for i in range(4)])

    asyncio.run(main())
    # strictly nested: in/out pairs never interleave
    for k in range(0, len(events), 2):
        assert events[k][0] == "in" and events[k + 1] == ("out", events[k][1])
    assert len(events) == 8
    # every acquire / release pair on one thread
    acq = [c for c in calls if c[0].endswith("lock") and "unlock" not in c[0]]
    rel = [c for c in calls if "unlock" in c[0]]
    assert len(acq) == len(rel) == 4
    assert {c[1] for c in calls} == {acq[0][1]}


def test_different_instances_do_not_block_each_other(instance_service):
    mod, _ = instance_service
    order = []

    async def hold(i, t):
        async with mod.InstanceLockAsync(types.SimpleNamespace(id=i)):
            order.append(("in", i))
            await asyncio.sleep(t)
            order.append(("out", i))

    async def main():
        await asyncio.gather(hold(1, 0.05), hold(2, 0.0))

    asyncio.run(main())
    assert order.index(("in", 2)) < order.index(("out", 1))


def test_sync_lock_serialises_threads(instance_service):
    mod, _ = instance_service
    inst = types.SimpleNamespace(id=99)
    inside = []
    overlap = []

    def worker():
        for _ in range(20):
            with mod.InstanceLock(inst):
                inside.append(1)
                if len(inside) > 1:
                    overlap.append(True)
                inside.pop()

    ts = [threading.Thread(target=worker) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not overlap


def test_cancelled_acquire_releases_the_session_lock(instance_service):
    """a coroutine cancelled while the thread-sensitive worker is still inside
    pg_advisory_lock must not leak that session lock: the acquire completes, is released on the
    same thread, the in-process key lock is dropped, and CancelledError still reaches the caller."""
    mod, calls = instance_service
    inst = types.SimpleNamespace(id=7)
    real = mod.BaseInstanceLock._db_acquire

    def slow_acquire(self):
        import time

        time.sleep(0.2)
        real(self)

    mod.BaseInstanceLock._db_acquire = slow_acquire
    try:
        async def main():
            task = asyncio.ensure_future(mod.InstanceLockAsync(inst).__aenter__())
            await asyncio.sleep(0.05)
            task.cancel()
            with pytest.raises(asyncio.CancelledError):
                await task
            # the key lock is free again: a new holder gets through at once
            async with mod.InstanceLockAsync(inst):
                pass

        asyncio.run(main())
    finally:
        mod.BaseInstanceLock._db_acquire = real
    names = [c[0] for c in calls]
    assert names == ["SELECT pg_advisory_lock", "SELECT pg_advisory_unlock"] * 2
    assert calls[0][1] == calls[1][1]
