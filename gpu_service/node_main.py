"""gpu_service over all GPUs of a node as ONE process group (``django_assistant_bot_amd.parallel.node``).

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --max-restarts 3 \\
        --master-addr 127.0.0.1 -m gpu_service.node_main --port 11435

Layout from the settings / environment (``assistant.conf``): ``INDEX_SHARDS`` (0 = every GPU),
``EMBED_DP`` (0 = every GPU), ``GEN_TP`` (generator tensor-parallel degree; the node runs
world / GEN_TP replicas).  Models: ``GPU_SERVICE_EMBEDDERS`` / ``GPU_SERVICE_PROVIDERS``.

Rank 0 serves the FastAPI app of ``gpu_service.main`` (same endpoints) with the node facades swapped
in; ranks 1..N-1 run the command loop.  ``--max-restarts`` makes a rank fault restart the group (new
RCCL communicators) instead of hanging it.  The reference had no multi-GPU mode
(/root/reference/gpu_service/gunicorn_conf.py:9: N copies of one process on one device).
"""
from __future__ import annotations

import argparse
import logging
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

logger = logging.getLogger("gpu_service.node")


def _llm_kwargs(device_type: str, max_batch: int | None, checkpoint: str | None) -> dict:
    from django_assistant_bot_amd.engine.serving import setting

    kw = {"block_size": setting("KV_BLOCK_SIZE", 64), "max_prefill_tokens": setting("MAX_BATCH_TOKENS", 65536),
          "max_batch": max_batch or (64 if device_type == "cuda" else 4)}
    if device_type != "cuda":
        kw.update(max_model_len=2048, use_graphs=False)
    if checkpoint:
        kw["checkpoint"] = checkpoint
    return kw


def setup(embedders=None, providers=None, plan=None, max_batch=None, checkpoint=None, backend=None,
          device_type=None, seed: int = 0, llm_weights=None):
    """Collective bootstrap on every rank: process group, node layout, engines.  On rank 0 the node
    facades are installed into the serving registry and gpu_service's index backend, so the FastAPI
    app serves the node.  Returns the ``Node``."""
    from django_assistant_bot_amd.engine import serving
    from django_assistant_bot_amd.parallel import dist as pdist
    from django_assistant_bot_amd.parallel.node import Node, NodeEmbedder, NodeIndexes, NodeLLM, NodePlan

    from gpu_service import main as svc
    from gpu_service import models as registry

    info = pdist.init(backend=backend, device_type=device_type)
    plan = plan or NodePlan.from_settings(info.world_size)
    embedders = registry.embedder_models if embedders is None else embedders
    providers = registry.provider_models if providers is None else providers
    node = Node(info, plan, embedders, providers, seed=seed,
                llm_kwargs=_llm_kwargs(info.device.type, max_batch, checkpoint), llm_weights=llm_weights)
    serving._node = node
    if info.rank == 0:
        for name in node.llms:
            serving._llm[name] = serving.LLMWorker(NodeLLM(node, name))
        for name in node.embeds:
            serving._emb[name] = serving.EmbedWorker(NodeEmbedder(node, name))
        svc.index_backend = NodeIndexes(node)
        svc.load_models(embedders, providers)  # providers / embedders pick up the node workers
    logger.info("rank %d: node plan %s (tp group rank %d, replica %d)", info.rank, plan, node.tp_rank, node.replica)
    return node


def exit_on_fault(node, grace_s: float = 2.0, poll_s: float = 0.5, exit=None):
    """Rank 0 watchdog: once the group is broken (a rank died, a collective failed), keep answering
    /health with 503 for ``grace_s`` and then leave with status 1, so ``torch.distributed.run
    --max-restarts`` restarts every rank with a fresh process group (new RCCL communicators)."""
    import threading
    import time

    def watch():
        while node.healthy:
            time.sleep(poll_s)
        logger.error("node group broken (%s); exiting for a restart", node.last_error)
        time.sleep(grace_s)
        (exit or os._exit)(1)

    t = threading.Thread(target=watch, name="node-watchdog", daemon=True)
    t.start()
    return t


def teardown(node) -> None:
    from django_assistant_bot_amd.engine import serving
    from django_assistant_bot_amd.parallel import dist as pdist

    if node.rank == 0:
        for w in list(serving._llm.values()) + list(serving._emb.values()):
            if hasattr(w, "stop"):
                w.stop()
        for w in serving._llm.values():
            w.join(60)  # a step in flight is a command: it must end before the stop broadcast
        node.shutdown()
    pdist.shutdown()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=11435)
    ap.add_argument("--max-batch", type=int, default=None)
    ap.add_argument("--checkpoint", default=None, help="HF safetensors dir of the generator (random-init if omitted)")
    a = ap.parse_args(argv)
    node = setup(max_batch=a.max_batch, checkpoint=a.checkpoint)
    if node.rank != 0:
        try:
            n = node.follow()
            logger.info("rank %d: %d commands, stopped", node.rank, n)
        finally:
            teardown(node)
        return 0
    import uvicorn

    from gpu_service.main import app

    exit_on_fault(node)
    try:
        uvicorn.run(app, host=a.host, port=a.port, log_level="info")
    finally:
        teardown(node)
    return 0


if __name__ == "__main__":
    sys.exit(main())
