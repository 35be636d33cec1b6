"""gpu_service with a tensor-parallel generator (e.g. Llama-3-70B over the 8 GPUs of one node).

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m gpu_service.tp_main --model llama-3-70b --port 11435

Every rank builds its shard of the engine (RCCL TP group over xGMI).  Rank 0 is the TP leader
(``django_assistant_bot_amd.parallel.tp_serving.TPLeader``).  It serves HTTP through the same
FastAPI app as ``gpu_service.main``, with embedders and indexes on GPU 0 only, and mirrors every
scheduler step to the followers.  Ranks 1..N-1 run ``follow()`` until the leader shuts down.
``GPU_SERVICE_PROVIDERS`` is set to the TP model, so /dialog/ serves it.  The reference served
no generator by default.
"""
from __future__ import annotations

import argparse
import logging
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

logger = logging.getLogger("gpu_service.tp")


def build_engine(model: str, info, tp_group, tp_rank: int, tp_size: int, **kw):
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine
    from django_assistant_bot_amd.engine.serving import setting

    kw.setdefault("max_batch", 64)
    kw.setdefault("block_size", setting("KV_BLOCK_SIZE", 64))
    kw.setdefault("max_prefill_tokens", setting("MAX_BATCH_TOKENS", 65536))
    return LLMEngine(model, info.device, tp_group=tp_group, tp_size=tp_size, tp_rank=tp_rank, **kw)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default=os.environ.get("GPU_SERVICE_TP_MODEL", "llama-3-70b"))
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=11435)
    ap.add_argument("--max-batch", type=int, default=64)
    ap.add_argument("--checkpoint", default=None, help="HF safetensors dir (random-init weights if omitted)")
    a = ap.parse_args(argv)

    from django_assistant_bot_amd.engine import serving
    from django_assistant_bot_amd.parallel import dist as pdist
    from django_assistant_bot_amd.parallel import tp_serving

    info = pdist.init()
    world = info.world_size
    tp_group, tp_rank, _ = pdist.tp_groups(world)
    ctrl = tp_serving.control_group(list(range(world))) if world > 1 else None
    engine = build_engine(a.model, info, tp_group, tp_rank, world, max_batch=a.max_batch, checkpoint=a.checkpoint)
    if info.rank != 0:
        steps = tp_serving.follow(engine, ctrl)
        logger.info("follower %d done after %d steps", info.rank, steps)
        pdist.shutdown()
        return 0
    leader = tp_serving.TPLeader(engine, ctrl) if world > 1 else engine
    serving._llm[a.model.lower()] = serving.LLMWorker(leader)  # picked up by the provider registry
    os.environ["GPU_SERVICE_PROVIDERS"] = a.model
    import uvicorn

    from gpu_service.main import app

    try:
        uvicorn.run(app, host=a.host, port=a.port, log_level="info")
    finally:
        worker = serving._llm[a.model.lower()]
        worker.stop()
        worker.join(60)  # its step (a control broadcast) must end before ours
        if world > 1:
            leader.shutdown()
        pdist.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
