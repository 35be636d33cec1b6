"""Celery ``shared_task`` when Celery is installed; otherwise an eager stand-in with the same
``.delay`` / ``.apply_async`` surface that runs the task inline (the equivalent of Celery's
``task_always_eager``).  Lets the Django-free core and the tests enqueue work without a broker."""
from __future__ import annotations

import functools
import logging

logger = logging.getLogger(__name__)

try:  # pragma: no cover - exercised where Celery is installed
    from celery import shared_task  # noqa: F401
    HAVE_CELERY = True
except ImportError:
    HAVE_CELERY = False

    class _EagerResult:
        def __init__(self, value=None, error=None):
            self.result, self.error = value, error

        def get(self, timeout=None):
            if self.error is not None:
                raise self.error
            return self.result

    def shared_task(fn=None, **options):
        def wrap(f):
            @functools.wraps(f)
            def task(*args, **kwargs):
                return f(*args, **kwargs)

            def apply_async(args=(), kwargs=None, **_):
                try:
                    return _EagerResult(f(*args, **(kwargs or {})))
                except Exception as e:  # Celery stores the failure on the result
                    logger.exception("eager task %s failed", f.__name__)
                    return _EagerResult(error=e)

            task.delay = lambda *a, **kw: apply_async(a, kw)
            task.apply_async = apply_async
            task.options = options
            return task
        return wrap(fn) if fn is not None else wrap
