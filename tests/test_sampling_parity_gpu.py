"""Sampling parity with HF ``generate`` at the real vocabulary size.

The reference samples with ``do_sample=True, top_k=50, top_p=0.95`` through HF's logits warpers
(/root/reference/assistant/ai/providers/transformers.py:62-64).  Here the oracle is HF itself:
``TemperatureLogitsWarper`` -> ``TopKLogitsWarper`` -> ``TopPLogitsWarper`` -> softmax over one
128,256-token logit row (the row the GPU reads, bf16-rounded).  The native samplers draw 300k tokens
from that same row (one row per draw, each with its own RNG counter; the rows are a stride-0 view,
so no copy is made) and the empirical distribution must be within total-variation distance 0.01 of
HF's, with exactly HF's support.  Paths: the one-pass exact sampler (``sample_tokens(fast=False)``),
the two-stage fast sampler (per-8192-chunk top-64, then merge), and the vocab-parallel pair
``sample_candidates`` (each TP rank's vocabulary slice) -> ``sample_merge`` at TP 2 and 8.
Cases: temperature 1.0 and 0.7 with the top-p cut inside the top 50; ties at the 50th logit
(HF keeps every logit >= the k-th value).  ``ops.reference.sample_hf`` against the same oracle:
tests/test_sampling_reference_cpu.py.
"""
import pytest
import torch

from django_assistant_bot_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
V = 128256
N_DRAWS = 300_000


def _row(kind: str) -> torch.Tensor:
    """A peaked logit row: 60 leading tokens at random positions, 0.125 apart (exact in bf16), over
    a background that top-k removes.  ``ties50``: ranks 47..52 share one value, so the 50th logit is
    tied with three more (HF keeps 53 tokens)."""
    g = torch.Generator().manual_seed(1234)
    x = (torch.randn(V, generator=g) * 1.5).clamp(max=3.0)
    pos = torch.randperm(V, generator=g)[:60]
    vals = 12.0 - 0.125 * torch.arange(60, dtype=torch.float32)
    if kind == "ties50":
        vals[47:53] = vals[47]
    x[pos] = vals
    return x.to(torch.bfloat16)


def _hf_probs(row_bf16: torch.Tensor, temp: float, top_k: int, top_p: float) -> torch.Tensor:
    from transformers.generation.logits_process import (TemperatureLogitsWarper, TopKLogitsWarper,
                                                        TopPLogitsWarper)

    x = row_bf16.float()[None].clone()
    if temp != 1.0:
        x = TemperatureLogitsWarper(temp)(None, x)
    x = TopKLogitsWarper(top_k=top_k)(None, x)
    if top_p < 1.0:
        x = TopPLogitsWarper(top_p=top_p)(None, x)
    return torch.softmax(x, -1)[0]


def _draw(path: str, row: torch.Tensor, temp: float, top_k: int, top_p: float, seed: int = 11) -> torch.Tensor:
    R = N_DRAWS
    logits = row.to(DEV)[None].expand(R, V)  # stride 0 over rows: every draw reads the same logits
    t = torch.full((R,), temp, device=DEV)
    k = torch.full((R,), top_k, dtype=torch.int32, device=DEV)
    p = torch.full((R,), top_p, device=DEV)
    cnt = torch.arange(R, dtype=torch.int64, device=DEV) * 7 + 3
    if path in ("exact", "fast"):
        return ops.sample_tokens(logits, t, k, p, seed, cnt, fast=(path == "fast")).long()
    tp = int(path[2:])
    Vs = V // tp
    parts = [ops.sample_candidates(logits[:, r * Vs:(r + 1) * Vs], Vs, r * Vs) for r in range(tp)]
    allc = torch.stack(parts, 2).reshape(2, R, -1).contiguous()  # what the TP all-gather assembles
    del parts
    return ops.sample_merge(allc, t, k, p, seed, cnt, V).long()


CASES = [("peaked", 1.0, 50, 0.95), ("peaked", 0.7, 50, 0.95), ("ties50", 1.0, 50, 1.0),
         ("ties50", 0.7, 50, 0.95)]


@pytest.mark.parametrize("path", ["exact", "fast", "tp2", "tp8"])
@pytest.mark.parametrize("case", CASES, ids=["t1", "t07", "ties", "ties_t07"])
def test_native_sampler_matches_hf_warpers(path, case):
    kind, temp, top_k, top_p = case
    row = _row(kind)
    want = _hf_probs(row, temp, top_k, top_p)
    support = set(torch.nonzero(want > 0).flatten().tolist())
    if kind == "ties50" and top_p == 1.0:
        assert len(support) == 53  # the tie at the 50th value extends HF's top-k set
    else:
        assert len(support) < 50  # the top-p cut falls inside the top 50
    tok = _draw(path, row, temp, top_k, top_p).cpu()
    freq = torch.bincount(tok, minlength=V).double() / tok.numel()
    drawn = set(torch.nonzero(freq > 0).flatten().tolist())
    assert drawn <= support, sorted(drawn - support)[:10]
    # every supported token with >= 2e-4 probability shows up (>= 60 expected draws each)
    assert {i for i in support if float(want[i]) >= 2e-4} <= drawn
    tv = 0.5 * float((freq - want.double()).abs().sum())
    assert tv <= 0.01, tv


def test_greedy_takes_the_lowest_index_among_tied_maxima():
    """torch.argmax semantics (HF greedy) on a row whose maximum is tied."""
    row = _row("peaked").float()
    top = int(row.argmax())
    other = (top + 5000) % V
    row[other] = row[top]
    lo = min(top, other)
    logits = row.to(torch.bfloat16).to(DEV)[None].expand(4, V)
    z = torch.zeros(4, device=DEV)
    k = torch.full((4,), 50, dtype=torch.int32, device=DEV)
    p = torch.ones(4, device=DEV)
    for fast in (False, True):
        cnt = torch.zeros(4, dtype=torch.int64, device=DEV)
        got = ops.sample_tokens(logits, z, k, p, 1, cnt, fast=fast)
        assert got.tolist() == [lo] * 4, (fast, got.tolist(), lo)


@pytest.mark.parametrize("path", ["exact", "fast", "tp2"])
def test_masked_row_with_fewer_allowed_tokens_than_top_k(path):
    """A constrained-decoding row (mask_logits: -inf outside the allowed set) with 3 allowed tokens
    and top-k 50: the -inf logits tie at the k-th value, carry probability 0 and are never drawn (nor
    walked: the tie extension stops at -inf); the draw follows softmax over the 3 allowed logits."""
    row = torch.full((V,), float("-inf"))
    allowed = torch.tensor([17, 70_000, 128_000])
    row[allowed] = torch.tensor([1.0, 0.5, 0.0])
    row = row.to(torch.bfloat16)
    want = torch.softmax(row.float()[allowed], 0)
    tok = _draw(path, row, 1.0, 50, 1.0).cpu()
    assert set(tok.unique().tolist()) <= set(allowed.tolist())
    freq = torch.stack([(tok == a).double().mean() for a in allowed.tolist()])
    assert float((freq - want.double()).abs().max()) < 0.01, (freq, want)
