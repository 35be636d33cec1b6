"""SURVEY.md 5.3 failure model of the node service on CPU gloo ranks: a rank that fails inside a
command breaks the group; rank 0 detects it on its next command (NodeFault, /health 503) and exits;
``torch.distributed.run --max-restarts`` restarts every rank with a new process group, which then
serves again."""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rank_fault_restarts_the_group(tmp_path):
    out = str(tmp_path / "res.txt")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--max-restarts", "1", "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "progs", "node_restart_prog.py"), out]
    env = dict(os.environ, OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               GPU_SERVICE_DEVICE="cpu")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    assert open(out + ".attempt0").read() == "detected healthy=False"
    assert open(out).read() == "recovered attempt=1 top=[0, 1]"
