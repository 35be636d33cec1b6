"""Auto-reload of the developer commands without Django (assistant/utils/autoreload.py): a child
process runs the command; editing a loaded source file restarts it; a normal exit ends the parent."""
import subprocess
import sys
import textwrap
import time


def test_reloader_restarts_child_on_source_change(tmp_path):
    log = tmp_path / "log.txt"
    mod = tmp_path / "helper_mod.py"
    mod.write_text("VALUE = 1\n")
    script = tmp_path / "prog.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys, time
        sys.path.insert(0, {str(tmp_path)!r})
        sys.path.insert(0, {sys.path[0]!r})
        import helper_mod
        from assistant.utils.autoreload import run_with_reloader

        def main(tag):
            with open({str(log)!r}, "a") as f:
                f.write(f"start {{tag}} {{helper_mod.VALUE}}\\n")
            if helper_mod.VALUE == 2:
                return  # the reloaded code finishes: the parent exits with 0
            time.sleep(30)

        sys.exit(run_with_reloader(main, "x", interval=0.2, use_django=False))
    """))
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.Popen([sys.executable, str(script)], cwd=root,
                         env={**os.environ, "PYTHONPATH": root, "PYTHONDONTWRITEBYTECODE": "1"})
    try:
        t0 = time.time()
        while not (log.exists() and log.read_text().count("start") >= 1):
            assert time.time() - t0 < 60, "child never started"
            time.sleep(0.1)
        time.sleep(0.5)
        mod.write_text("VALUE = 2\n")
        rc = p.wait(timeout=60)
    finally:
        if p.poll() is None:
            p.kill()
    assert rc == 0
    assert log.read_text().splitlines() == ["start x 1", "start x 2"]
