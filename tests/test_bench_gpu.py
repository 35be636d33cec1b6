"""bench.py on the GPU path with the tiny presets: batch, serve and overlap modes in one process
(HIP-graph decode, native kernels), and the 2-rank launch shape of ``torch.distributed.run`` with both
ranks on the one GPU (gloo: RCCL needs a device per rank).  Each run prints exactly one JSON line
with the driver's keys and a positive whole-job value."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--embed-model", "tiny-bert", "--llm-model", "tiny-llama", "--index-rows", "20000", "--batch", "8",
        "--max-new-tokens", "8", "--steps", "1", "--warmup", "1"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd, **env):
    p = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ, **env), capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["dtype"] == "bf16"
    return d


@pytest.mark.parametrize("mode", ["batch", "serve", "overlap", "qps"])
def test_bench_modes_on_gpu(mode):
    args = list(TINY)
    if mode == "qps":  # open loop: a fixed arrival schedule (profiles/fixed_qps.md)
        mode, args = "serve", args + ["--qps", "20"]
    if mode == "overlap":
        args[args.index("--steps") + 1] = "2"
        args[args.index("--warmup") + 1] = "2"
    d = _run([sys.executable, "bench.py", "--mode", mode, *args])
    assert d["config"]["mode"].startswith(mode) and d["config"]["graphs"] is True
    assert d["n_gpus"] == 1


@pytest.mark.parametrize("tp", [1, 2])
def test_bench_two_ranks_on_one_gpu(tp):
    """tp 1: two DP replicas with the index sharded over them; tp 2: one TP-2 generator (IPC
    all-reduce inside the decode graphs) -- config 5's launch shape at toy size."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2", "--tp", str(tp)] + TINY
    d = _run(cmd, DAB_DIST_BACKEND="gloo")
    assert d["n_gpus"] == 2
    if tp == 1:
        assert d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 16
    else:
        assert "tp2" in d["config"]["parallelism"]


def test_bench_four_ranks_on_one_gpu():
    """The multi-GPU launch shape at 4 ranks (index sharded 4 ways, all_to_all merge), on one card."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "4"] + TINY
    d = _run(cmd, DAB_DIST_BACKEND="gloo")
    assert d["n_gpus"] == 4 and d["config"]["parallelism"] == "dp4" and d["config"]["global_batch"] == 32


def test_bench_self_launches_four_ranks_on_one_gpu():
    """The driver's form ``python bench.py --gpus 4`` as ONE plain command: bench.py starts the four
    ranks itself (parallel/launch.py) and reports the world that formed (gloo: all on one card)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["DAB_DIST_BACKEND"] = "gloo"
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "4", *TINY], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["backend"] == "gloo" and len(d["config"]["per_rank_qps"]) == 4
    assert d["config"]["parallelism"] == "dp4" and d["value"] > 0


def test_bench_config5_eight_rank_rehearsal():
    """BASELINE config 5 as one command, ``bench.py --config 5 --gpus 8``: bge-large retriever and
    Llama-3-70B's attention layout (hidden 8192, 64 / 8 heads of D = 128) at 2 layers with TP = 8,
    open-loop serve at a fixed QPS -- 8 ranks on the one card over gloo, IPC all-reduce in the graphs."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["DAB_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, "bench.py", "--config", "5", "--gpus", "8", "--llm-model", "tiny-llama-70b-d128",
           "--index-rows", "20000", "--batch", "8", "--max-new-tokens", "8", "--qps", "20", "--steps", "1",
           "--warmup", "1", "--no-fast-steps"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    if p.returncode:  # the launcher's summary ends stderr: keep the ranks' own tracebacks too
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", "config5_rehearsal.stderr"), "w") as f:
            f.write(p.stderr)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["config"]["parallelism"] == "dp1xtp8" and "70B" in d["metric"]
    assert d["config"]["model"] == "bge-large-en + tiny-llama-70b-d128"
    assert d["value"] > 0 and d["config"]["graphs"] is True
