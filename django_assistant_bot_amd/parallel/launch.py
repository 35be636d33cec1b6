"""Self-launch of N ranks for the benchmarks (``bench.py --gpus N`` run as a plain process).

The reference's only scaling knob is a worker count it spawns itself (gunicorn ``workers = 2``,
/root/reference/gpu_service/gunicorn_conf.py:9).  The engine's scaling unit is one process per GPU
over RCCL, so a benchmark asked for N GPUs starts those N processes itself when it is not already
one rank of a ``torch.distributed.run`` job:

* the parent never touches the GPU (it only imports torch and counts nothing), so no HIP state
  exists in the process that spawns the workers, and the workers are children, not an ``exec``;
* rank 0's stdout (the one JSON line) is forwarded as it arrives; every worker's stderr goes to
  the parent's stderr;
* the parent exits with the first non-zero worker exit code, or 0.

Inside a worker, :func:`check_world` turns a mismatch between ``--gpus`` and the group that formed
into a hard error.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def in_launched_job() -> bool:
    """True when this process is one rank of a torch.distributed.run (or equivalent) job."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def spawn_ranks(n: int, script: str, argv: list[str], max_restarts: int = 0) -> int:
    """Run ``script argv`` as ``n`` ranks of one node (torch.distributed.run, rendezvous on
    127.0.0.1) and return the job's exit code.  Output of rank 0 is passed through unchanged."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "--max-restarts", str(max_restarts), script, *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    env["DAB_SPAWNED_BY_PARENT"] = "1"
    # without --tee / --redirects torchrun leaves the ranks' stdout inherited, and only rank 0 prints
    # the JSON line, so the parent's stdout carries exactly that line
    proc = subprocess.Popen(cmd, env=env, stdout=sys.stdout, stderr=sys.stderr)
    try:
        return proc.wait()
    except KeyboardInterrupt:
        proc.terminate()
        return proc.wait()


def maybe_spawn(n_gpus: int, script: str, argv: list[str] | None = None) -> None:
    """If ``n_gpus > 1`` and this process is not already a rank, launch the N-rank job and exit
    with its code (never returns then).  Otherwise return and let the caller run as a rank."""
    if n_gpus <= 1 or in_launched_job():
        return
    code = spawn_ranks(n_gpus, os.path.abspath(script), list(sys.argv[1:] if argv is None else argv))
    sys.exit(code)


def check_world(requested: int, formed: int) -> None:
    """Hard error when the process group that formed is not the one ``--gpus`` asked for."""
    if requested != formed:
        raise SystemExit(f"--gpus {requested} but the job formed a world of {formed} ranks "
                         f"(WORLD_SIZE={os.environ.get('WORLD_SIZE')}); refusing to report a mislabelled result")
