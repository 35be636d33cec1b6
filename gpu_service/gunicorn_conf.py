"""Gunicorn config (reference gpu_service/gunicorn_conf.py).

One worker process per GPU: each worker is pinned to the lowest device no live worker holds
(``pre_fork`` runs in the arbiter, which knows the live workers; ``post_fork`` sets
HIP_VISIBLE_DEVICES before the worker imports torch), so a respawned worker takes over exactly the
GPU its predecessor left.  The workers are independent replicas for /embeddings/ and /dialog/; one
index over all GPUs (and DP / TP engines) is node mode: ``gpu_service/node_main.py``.  The
reference ran GPU_SERVICE_WORKERS copies on one device."""
import os

bind = os.environ.get("GPU_SERVICE_BIND", "0.0.0.0:11435")
devices = int(os.environ.get("GPU_SERVICE_DEVICES", "1"))
workers = int(os.environ.get("GPU_SERVICE_WORKERS", str(devices)))
worker_class = "uvicorn.workers.UvicornWorker"
timeout = int(os.environ.get("GPU_SERVICE_TIMEOUT", "120"))
accesslog = os.environ.get("GPU_SERVICE_ACCESS_LOG", "-")
errorlog = os.environ.get("GPU_SERVICE_ERROR_LOG", "-")
loglevel = os.environ.get("GPU_SERVICE_LOG_LEVEL", "info")
raw_env = ["TOKENIZERS_PARALLELISM=false", "HSA_ENABLE_IPC_MODE_LEGACY=0", f"GPU_SERVICE_WORKERS={workers}"]
preload_app = False  # each worker initialises its own GPU


def pick_device(live_workers, n_devices: int) -> int:
    """Lowest device index not held by a live worker (workers beyond the device count share round-robin)."""
    held = [getattr(w, "dab_device", None) for w in live_workers]
    n = max(n_devices, 1)
    for d in range(n):
        if d not in held:
            return d
    return min(range(n), key=lambda d: (held.count(d), d))


def pre_fork(server, worker):
    others = [w for w in server.WORKERS.values() if w is not worker]
    worker.dab_device = pick_device(others, devices)


def post_fork(server, worker):
    dev = getattr(worker, "dab_device", 0)
    os.environ["HIP_VISIBLE_DEVICES"] = str(dev)
    server.log.info("worker %s -> GPU %s", worker.pid, dev)
