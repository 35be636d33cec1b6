"""Model-level GPU checks: the decode step through the weight-streaming split-K GEMM (slab-summing
RoPE / RMSNorm consumers, fused SwiGLU, skinny LM head) against the same model on the hipBLASLt
path and against the fp32 CPU reference."""
import pytest
import torch

from django_assistant_bot_amd import ops
from django_assistant_bot_amd.models.configs import decoder_config
from django_assistant_bot_amd.models.llama import AttnMeta, KVCache, LlamaModel
from django_assistant_bot_amd.models.weights import random_decoder_weights

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(model, cfg, prompts, device, dtype):
    bs, nb_per = 64, 4
    B = len(prompts)
    kv = KVCache(cfg.layers, B * nb_per, cfg.kv_heads, bs, cfg.head_dim, device, dtype=dtype)
    bt = torch.arange(B * nb_per, dtype=torch.int32, device=device).view(B, nb_per)
    for b, ids in enumerate(prompts):  # prefill each prompt but its last token
        T = len(ids) - 1
        meta = AttnMeta(decode=False, positions=torch.arange(T, dtype=torch.int32, device=device),
                        slots=(bt[b, 0].long() * bs + torch.arange(T, device=device)),
                        block_tables=bt[b:b + 1], ctx_lens=torch.tensor([T], dtype=torch.int32, device=device),
                        cu_q=torch.tensor([0, T], dtype=torch.int32, device=device), max_q=T)
        model.forward(torch.tensor(ids[:-1], dtype=torch.int32, device=device), meta, kv)
    pos = torch.tensor([len(p) - 1 for p in prompts], dtype=torch.int32, device=device)
    slots = bt[:, 0].long() * bs + pos.long()
    ws = ops.DecodeWorkspace(B, cfg.heads, cfg.head_dim, nb_per * bs // 512 + 1, device) if device != "cpu" else None
    meta = AttnMeta(decode=True, positions=pos, slots=slots, block_tables=bt, ctx_lens=pos + 1, workspace=ws)
    h = model.forward(torch.tensor([p[-1] for p in prompts], dtype=torch.int32, device=device), meta, kv)
    return h, model.logits(h)


@pytest.mark.parametrize("B", [3, 20, 64])
def test_decode_skinny_matches_library_path_and_reference(B):
    cfg = decoder_config("tiny-llama")
    w32 = random_decoder_weights(cfg, dtype=torch.float32, seed=5, interleave_mlp=True)
    gen = torch.Generator().manual_seed(B)
    prompts = [torch.randint(0, cfg.vocab_size, (int(n),), generator=gen).tolist()
               for n in torch.randint(10, 150, (B,), generator=gen)]
    wbf = {k: v.to(torch.bfloat16) for k, v in w32.items()}
    m_sk = LlamaModel(cfg, wbf, DEV, interleaved_mlp=True)
    m_sk.skinny_for = {"qkv", "o", "gate_up", "down", "lm_head"}  # every decode projection
    m_sk.use_skinny = True
    h_sk, lg_sk = _run(m_sk, cfg, prompts, DEV, torch.bfloat16)
    m_lib = LlamaModel(cfg, wbf, DEV, interleaved_mlp=True)
    m_lib.use_skinny = False
    h_lib, lg_lib = _run(m_lib, cfg, prompts, DEV, torch.bfloat16)
    torch.testing.assert_close(h_sk.float(), h_lib.float(), atol=6e-2, rtol=5e-2)
    torch.testing.assert_close(lg_sk.float(), lg_lib.float(), atol=6e-2, rtol=5e-2)
    m_ref = LlamaModel(cfg, {k: v.bfloat16().float() for k, v in w32.items()}, "cpu", interleaved_mlp=True)
    h_ref, _ = _run(m_ref, cfg, prompts, "cpu", torch.float32)
    err = (h_sk.float().cpu() - h_ref).abs().max().item()
    assert err < 0.15, err
