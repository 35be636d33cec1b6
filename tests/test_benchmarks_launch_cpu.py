"""The config-2 and config-3 benchmarks start their own ranks for ``--gpus N`` (parallel/launch.py),
like bench.py: one plain command, rank 0's JSON line, ``n_gpus`` = the world that formed."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_embed_bench_self_launch_two_ranks():
    d = _run([sys.executable, "benchmarks/embed_bench.py", "--gpus", "2", "--model", "tiny-bert", "--chunks", "600",
              "--warmup-chunks", "50", "--words", "12"])
    assert d["n_gpus"] == 2 and d["chunks"] == 600 and d["value"] > 0 and d["config"]["parallelism"] == "dp2"


def test_index_bench_self_launch_two_ranks():
    d = _run([sys.executable, "benchmarks/index_bench.py", "--gpus", "2", "--rows", "20000", "--dim", "64",
              "--k", "16", "--batch", "1", "4", "--iters", "2", "--warmup", "1"])
    assert d["n_gpus"] == 2 and [r["queries_per_rank"] for r in d["results"]] == [1, 4]
