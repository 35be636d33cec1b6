"""Code auto-reload for the developer commands (``chat``, ``telegram_poll --dev``).

Inside a Django project this is ``django.utils.autoreload.run_with_reloader`` (what the reference
commands call: bot/management/commands/chat.py:47-48, telegram_poll.py:31,46).  Without Django the
same protocol is implemented here: the launching process starts the command again as a child with
``DAB_RELOADER_CHILD=true``; the child runs ``main`` while a watcher thread polls the modification
times of every loaded Python module (and the entry script); on a change the child exits with code 3
and the parent starts a fresh child.  Any other exit code ends the parent with that code.  The child
is a new process (subprocess), never an exec of the running one.
"""
from __future__ import annotations

import os
import subprocess
import sys
import threading
import time

CHILD_FLAG = "DAB_RELOADER_CHILD"
RELOAD_EXIT = 3


def watched_files() -> set[str]:
    files = set()
    for mod in list(sys.modules.values()):
        f = getattr(mod, "__file__", None)
        if f and f.endswith(".py") and os.path.exists(f):
            files.add(os.path.abspath(f))
    if sys.argv and sys.argv[0].endswith(".py") and os.path.exists(sys.argv[0]):
        files.add(os.path.abspath(sys.argv[0]))
    return files


def _mtimes(files) -> dict:
    out = {}
    for f in files:
        try:
            out[f] = os.stat(f).st_mtime_ns
        except OSError:
            out[f] = None
    return out


def _watch(interval: float, on_change) -> None:
    seen = _mtimes(watched_files())
    while True:
        time.sleep(interval)
        files = watched_files()
        now = _mtimes(files)
        changed = [f for f in files if f in seen and now.get(f) != seen[f]]
        if changed:
            on_change(changed)
            return
        seen.update({f: t for f, t in now.items() if f not in seen})


def child_arguments() -> list[str]:
    """The command line that starts this program again (``python -m pkg.mod`` stays a module run)."""
    main_mod = sys.modules.get("__main__")
    spec = getattr(main_mod, "__spec__", None)
    if spec is not None and spec.name and spec.name != "__main__":
        name = spec.name[: -len(".__main__")] if spec.name.endswith(".__main__") else spec.name
        return [sys.executable, "-m", name] + sys.argv[1:]
    return [sys.executable] + sys.argv


def run_with_reloader(main, *args, interval: float = 1.0, use_django: bool = True, **kwargs):
    if use_django:
        try:
            from django.utils import autoreload as dj
        except ImportError:
            dj = None
        if dj is not None:
            return dj.run_with_reloader(main, *args, **kwargs)
    if os.environ.get(CHILD_FLAG) == "true":
        def changed(files):
            sys.stderr.write(f"{files[0]} changed, reloading.\n")
            sys.stderr.flush()
            os._exit(RELOAD_EXIT)

        threading.Thread(target=_watch, args=(interval, changed), name="autoreload", daemon=True).start()
        main(*args, **kwargs)
        return 0
    env = dict(os.environ, **{CHILD_FLAG: "true"})
    while True:
        try:
            rc = subprocess.call(child_arguments(), env=env)
        except KeyboardInterrupt:
            return 0
        if rc != RELOAD_EXIT:
            return rc
