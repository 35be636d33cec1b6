"""Launched by tests/test_node_fault.py under ``torch.distributed.run --max-restarts 1`` (gloo, CPU).

Attempt 0: rank 1 fails inside a command; rank 0's next command raises NodeFault, /health turns 503
and the watchdog exits the process, so the launcher restarts BOTH ranks.  Attempt 1: a fresh group
(new communicators) serves the index commands again; rank 0 records the outcome."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main(out_path: str) -> int:
    import torch

    torch.set_num_threads(1)
    from django_assistant_bot_amd.engine import serving
    from django_assistant_bot_amd.parallel.node import NodeFault, NodePlan
    from gpu_service import node_main

    attempt = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
    world = int(os.environ["WORLD_SIZE"])
    node = node_main.setup(embedders=[], providers=[], plan=NodePlan(world), backend="gloo", device_type="cpu")
    if node.rank != 0:
        try:
            node.follow()
        finally:
            node_main.teardown(node)
        return 0
    ids = np.arange(64)
    vecs = np.random.default_rng(0).standard_normal((64, 8)).astype(np.float32)
    n = node.command("index_upsert", ("t", ids, vecs, None, None))
    assert n == 64
    if attempt == 0:
        node.command("fault", 1)  # rank 1 dies inside this command
        t0 = time.time()
        try:
            while True:  # the next command notices the dead peer
                node.command("index_sizes", ["t"])
                assert time.time() - t0 < 60, "dead peer never detected"
                time.sleep(0.2)
        except NodeFault:
            pass
        with open(out_path + ".attempt0", "w") as f:
            f.write(f"detected healthy={serving.health()['healthy']}")
        node_main.exit_on_fault(node, grace_s=0.1, poll_s=0.05)
        time.sleep(30)  # the watchdog ends the process
        return 2
    sims, got, _ = node.command("index_search", ("t", vecs[:2], 3, None, None, None))
    with open(out_path, "w") as f:
        f.write(f"recovered attempt={attempt} top={got[:, 0].tolist()}")
    node_main.teardown(node)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
