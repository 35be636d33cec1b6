"""Inspect / clear / remove tasks of the Celery queues in the Redis broker (reference
admin/management/commands/queue.py).  Speaks the Redis protocol directly (no redis-py needed)."""
import socket
import urllib.parse

from django.core.management.base import BaseCommand, CommandError

from assistant.assistant.queue import CeleryQueues
from assistant.conf import settings


class RedisConnection:
    """Just enough RESP for LRANGE / DEL / LREM / SELECT."""

    def __init__(self, host: str, port: int, db: int = 0, password: str = None, timeout: float = 10.0):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.buf = b""
        if password:
            self.command("AUTH", password)
        if db:
            self.command("SELECT", db)

    def _readline(self) -> bytes:
        while b"\r\n" not in self.buf:
            chunk = self.sock.recv(65536)
            if not chunk:
                raise ConnectionError("redis closed the connection")
            self.buf += chunk
        line, self.buf = self.buf.split(b"\r\n", 1)
        return line

    def _read(self):
        line = self._readline()
        kind, rest = line[:1], line[1:]
        if kind == b"+":
            return rest.decode()
        if kind == b"-":
            raise CommandError(rest.decode())
        if kind == b":":
            return int(rest)
        if kind == b"$":
            n = int(rest)
            if n < 0:
                return None
            while len(self.buf) < n + 2:
                self.buf += self.sock.recv(65536)
            data, self.buf = self.buf[:n], self.buf[n + 2:]
            return data
        if kind == b"*":
            n = int(rest)
            return None if n < 0 else [self._read() for _ in range(n)]
        raise CommandError(f"bad redis reply {line!r}")

    def command(self, *args):
        parts = [str(a).encode() if not isinstance(a, bytes) else a for a in args]
        payload = b"*%d\r\n" % len(parts) + b"".join(b"$%d\r\n%s\r\n" % (len(p), p) for p in parts)
        self.sock.sendall(payload)
        return self._read()


class Command(BaseCommand):
    help = "Manage Celery queues in Redis"

    def add_arguments(self, parser):
        parser.add_argument("operation", choices=["list", "clear", "remove"])
        parser.add_argument("--name", choices=[q.value for q in CeleryQueues])
        parser.add_argument("--db", type=int, default=None, help="Redis DB (default: from the broker URL)")
        parser.add_argument("--task_id")

    def handle(self, *args, **opts):
        url = urllib.parse.urlparse(settings.CELERY_BROKER_URL)
        db = opts["db"] if opts["db"] is not None else int((url.path or "/0").lstrip("/") or 0)
        r = RedisConnection(url.hostname or "localhost", url.port or 6379, db, url.password)
        names = [opts["name"]] if opts["name"] else [q.value for q in CeleryQueues]
        op = opts["operation"]
        if op == "list":
            for name in names:
                for task in r.command("LRANGE", name, 0, -1) or []:
                    self.stdout.write(task.decode("utf-8", "replace"))
        elif op == "clear":
            for name in names:
                r.command("DEL", name)
                self.stdout.write(self.style.SUCCESS(f"Cleared queue `{name}`"))
        else:
            if not opts["task_id"] or not opts["name"]:
                raise CommandError("remove needs --name and --task_id")
            for task in r.command("LRANGE", opts["name"], 0, -1) or []:
                if opts["task_id"].encode() in task:
                    r.command("LREM", opts["name"], 1, task)
                    self.stdout.write(self.style.SUCCESS(f"Removed task {opts['task_id']}"))
                    return
            self.stdout.write(self.style.WARNING(f"Task {opts['task_id']} not found in {opts['name']}"))
