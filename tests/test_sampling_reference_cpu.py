"""``ops.reference.sample_hf`` -- the CPU oracle of the CPU test-suite -- against HF's own logits
warpers (TemperatureLogitsWarper -> TopKLogitsWarper -> TopPLogitsWarper), the sampling of the
reference (/root/reference/assistant/ai/providers/transformers.py:62-64).  A 4,096-token row keeps
the per-row Python oracle fast; the GPU samplers are checked at 128,256 tokens in
tests/test_sampling_parity_gpu.py."""
import torch

from django_assistant_bot_amd.ops import reference as ref


def _row(V=4096, ties=False):
    g = torch.Generator().manual_seed(77)
    x = (torch.randn(V, generator=g) * 1.5).clamp(max=3.0)
    pos = torch.randperm(V, generator=g)[:60]
    vals = 12.0 - 0.125 * torch.arange(60, dtype=torch.float32)
    if ties:
        vals[47:53] = vals[47]
    x[pos] = vals
    return x.to(torch.bfloat16).float()


def _hf(row, temp, k, p):
    from transformers.generation.logits_process import (TemperatureLogitsWarper, TopKLogitsWarper,
                                                        TopPLogitsWarper)

    x = row[None].clone()
    if temp != 1.0:
        x = TemperatureLogitsWarper(temp)(None, x)
    x = TopKLogitsWarper(top_k=k)(None, x)
    if p < 1.0:
        x = TopPLogitsWarper(top_p=p)(None, x)
    return torch.softmax(x, -1)[0]


def test_reference_sampler_matches_hf_warpers():
    for ties, temp, k, p in ((False, 1.0, 50, 0.95), (True, 0.7, 50, 0.95), (True, 1.0, 50, 1.0)):
        row = _row(ties=ties)
        want = _hf(row, temp, k, p)
        R = 20000
        g = torch.Generator().manual_seed(5)
        tok = ref.sample_hf(row[None].expand(R, -1), torch.full((R,), temp), torch.full((R,), k),
                            torch.full((R,), p), g).long()
        freq = torch.bincount(tok, minlength=row.numel()).double() / R
        assert set(torch.nonzero(freq > 0).flatten().tolist()) <= set(torch.nonzero(want > 0).flatten().tolist())
        assert 0.5 * float((freq - want.double()).abs().sum()) <= 0.03, (ties, temp, k, p)
        if ties and p == 1.0:
            assert int((want > 0).sum()) == 53  # HF keeps the logits tied with the 50th
