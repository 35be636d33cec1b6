"""Tracing helpers: roctx ranges through the native binding, GPU phase spans from HIP events."""
import pytest
import torch

from django_assistant_bot_amd.ops._lib import native
from django_assistant_bot_amd.utils import trace


def test_roctx_ranges_nest_and_are_noops_when_disabled():
    n = native()
    trace.set_roctx(False)
    with trace.range("off"):
        pass
    if not n.roctx_available():
        pytest.skip("roctx library not installed")
    trace.set_roctx(True)
    try:
        depth0 = n.roctx_push("outer")
        with trace.range("inner"):
            assert n.roctx_push("probe") == depth0 + 2
            n.roctx_pop()
        assert n.roctx_pop() == depth0
        trace.mark("point")
    finally:
        trace.set_roctx(False)


def test_gpu_timer_disabled_on_cpu():
    t = trace.GpuTimer(device="cpu")
    assert not t.enabled
    with t.phase("x"):
        torch.ones(3).sum()
    assert t.collect() == {}


@pytest.mark.gpu
def test_gpu_timer_spans():
    t = trace.GpuTimer(device="cuda")
    a = torch.randn(2048, 2048, device="cuda", dtype=torch.bfloat16)
    with t.phase("mm"):
        for _ in range(10):
            a = a @ a * 0.01
    with t.phase("mm"):
        a = a @ a
    out = t.collect()
    assert out["mm"] > 0 and t.counts["mm"] == 2


@pytest.mark.gpu
def test_engine_reports_gpu_phase_times():
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine, SamplingParams

    eng = LLMEngine("tiny-llama", device="cuda", max_batch=4, num_blocks=32)
    eng.generate([list(range(5, 40))] * 3, SamplingParams(max_new_tokens=6, ignore_eos=True))
    assert eng.stats["gpu_prefill_ms"] > 0 and eng.stats["gpu_decode_ms"] > 0
