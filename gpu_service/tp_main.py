"""gpu_service with one tensor-parallel generator over the whole node (e.g. Llama-3-70B on 8 GPUs):
node mode (``gpu_service.node_main``) with ``GEN_TP`` = world size.

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m gpu_service.tp_main --model llama-3-70b --port 11435
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default=os.environ.get("GPU_SERVICE_TP_MODEL", "llama-3-70b"))
    a, rest = ap.parse_known_args(argv)
    os.environ["GPU_SERVICE_PROVIDERS"] = a.model
    os.environ["GEN_TP"] = os.environ.get("WORLD_SIZE", "1")
    from gpu_service import node_main

    return node_main.main(rest)


if __name__ == "__main__":
    sys.exit(main())
