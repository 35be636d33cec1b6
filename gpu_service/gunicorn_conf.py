"""Gunicorn config (reference gpu_service/gunicorn_conf.py).

One worker process per GPU: worker i pins itself to device i % GPU_SERVICE_DEVICES (HIP_VISIBLE_DEVICES
set in post_fork, before the worker imports torch), so N GPUs serve N independent engine replicas
(data parallel) behind one port.  The reference ran GPU_SERVICE_WORKERS copies on one device."""
import os

bind = os.environ.get("GPU_SERVICE_BIND", "0.0.0.0:11435")
devices = int(os.environ.get("GPU_SERVICE_DEVICES", "1"))
workers = int(os.environ.get("GPU_SERVICE_WORKERS", str(devices)))
worker_class = "uvicorn.workers.UvicornWorker"
timeout = int(os.environ.get("GPU_SERVICE_TIMEOUT", "120"))
accesslog = os.environ.get("GPU_SERVICE_ACCESS_LOG", "-")
errorlog = os.environ.get("GPU_SERVICE_ERROR_LOG", "-")
loglevel = os.environ.get("GPU_SERVICE_LOG_LEVEL", "info")
raw_env = ["TOKENIZERS_PARALLELISM=false", "HSA_ENABLE_IPC_MODE_LEGACY=0"]
preload_app = False  # each worker initialises its own GPU


def post_fork(server, worker):
    dev = (worker.age - 1) % max(devices, 1)
    os.environ["HIP_VISIBLE_DEVICES"] = str(dev)
    server.log.info("worker %s -> GPU %s", worker.pid, dev)
