"""The bench.py driver contract on CPU: one rank and two gloo ranks (the multi-GPU launch shape of
``torch.distributed.run``) on the tiny model presets print exactly one JSON line with the required
keys, the whole-job aggregate and the data-parallel config."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}
TINY = ["--embed-model", "tiny-bert", "--llm-model", "tiny-llama", "--index-rows", "5000", "--batch", "4",
        "--max-new-tokens", "6", "--steps", "1", "--warmup", "1"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def _check(d, n):
    assert REQUIRED <= set(d)
    assert d["n_gpus"] == n and d["steps"] == 1 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["dtype"] == "bf16"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # the fast JSON steps (classify + known question) reported next to the unchanged headline
    assert d["fast_steps_s"] > 0 and 0 < d["full_pipeline_qps"] < d["value"]
    assert d["full_pipeline_p50_latency_ms"] > d["p50_latency_ms"]
    f = d["config"]["fast_steps"]
    assert f["batch"] == 4 and f["classify_prompt_tokens"] > 100 and f["known_question_prompt_tokens"] > 50
    c = d["config"]
    assert c["parallelism"] == f"dp{n}" and c["global_batch"] == 4 * n
    # whole-job aggregate: n replicas x batch 4 answered in the timed step
    assert d["value"] == pytest.approx(4 * n / (d["ms_per_step"] / 1000.0), rel=0.02)
    assert c["docs_per_prompt"] > 0


def test_bench_single_rank():
    _check(_run([sys.executable, "bench.py"] + TINY), 1)


def test_bench_two_gloo_ranks():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2"] + TINY
    _check(_run(cmd), 2)


def test_bench_self_launches_its_ranks():
    """``python bench.py --gpus 2`` as ONE plain command (the driver's form): the script starts the
    two ranks itself and the JSON reports the world that formed, its backend and per-rank rates."""
    d = _run([sys.executable, "bench.py", "--gpus", "2"] + TINY)
    _check(d, 2)
    assert d["backend"] == "gloo" and len(d["config"]["per_rank_qps"]) == 2


def test_bench_world_mismatch_is_an_error():
    """A torchrun world that is not the --gpus asked for fails instead of reporting a mislabelled number."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "4"] + TINY
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0 and "formed a world of 2" in p.stderr


def test_bench_config5_preset_self_launch():
    """--config 5 (Llama-3-70B layout TP = --gpus + bge-large, open-loop serve at a fixed QPS) at
    toy depth: 2 ranks form one TP-2 replica."""
    args = list(TINY)
    args[args.index("--llm-model") + 1] = "tiny-llama-70b-layout"
    d = _run([sys.executable, "bench.py", "--config", "5", "--gpus", "2", "--qps", "40", *args])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp1xtp2"
    assert d["config"]["mode"].startswith("serve (open loop") and d["vs_baseline"] is None
    assert "70B" in d["metric"] and d["value"] > 0


def test_bench_overlap_mode_single_process():
    """--mode overlap: two engines sharing one weight copy, each on its own thread / stream, batches
    alternating; the timed region answers every question once (2 timed batches of 4)."""
    args = [a for a in TINY]
    args[args.index("--steps") + 1] = "2"
    args[args.index("--warmup") + 1] = "2"
    d = _run([sys.executable, "bench.py", "--gpus", "1", "--mode", "overlap", *args])
    assert d["steps"] == 2 and d["value"] > 0 and d["config"]["mode"].startswith("overlap")
    assert d["value"] == pytest.approx(8 / (2 * d["ms_per_step"] / 1000.0), rel=0.02)
