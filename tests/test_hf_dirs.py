"""A local HF checkpoint directory as the model name (what the reference's TransformersEmbedder /
TransformersProvider accept: ``from_pretrained(model_name)``, ai/embedders/transformers.py:13,
ai/providers/transformers.py:18-20).  The architecture is read from config.json, the weights from
the safetensors files, the tokenizer from tokenizer.json: a ``save_pretrained`` HF Llama / BERT runs
on the engines with no preset.  Parity against the HF models themselves (fp32, CPU)."""
import json
import os
import shutil

import pytest
import torch

transformers = pytest.importorskip("transformers")


def _llama_dir(tmp, bpe_dir, rope_scaling=None, hidden=256, heads=4, kv_heads=2, tie=False):
    torch.manual_seed(0)
    hc = transformers.LlamaConfig(vocab_size=1024, hidden_size=hidden, num_hidden_layers=2, num_attention_heads=heads,
                                  num_key_value_heads=kv_heads, intermediate_size=512, rms_norm_eps=1e-5,
                                  rope_theta=500000.0, max_position_embeddings=2048, tie_word_embeddings=tie,
                                  bos_token_id=1000, eos_token_id=1001, rope_scaling=rope_scaling,
                                  attn_implementation="eager")
    hf = transformers.LlamaForCausalLM(hc).eval()
    with torch.no_grad():  # larger weights than the HF init: logits with clear argmaxes
        for p in hf.parameters():
            if p.ndim == 2:
                p.normal_(0.0, 0.08)
    d = os.path.join(tmp, "my-llama")
    hf.save_pretrained(d, safe_serialization=True)
    for f in os.listdir(bpe_dir):
        if f.startswith("tokenizer") or f.startswith("special"):
            shutil.copy(os.path.join(bpe_dir, f), d)
    return hf, d


LLAMA3_SCALING = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                  "original_max_position_embeddings": 256}


def test_decoder_config_from_hf_dir(tmp_path, bpe_dir):
    from django_assistant_bot_amd.models.configs import decoder_config, is_decoder, is_encoder

    _, d = _llama_dir(str(tmp_path), bpe_dir, rope_scaling=LLAMA3_SCALING)
    cfg = decoder_config(d)
    assert (cfg.name, cfg.vocab_size, cfg.hidden, cfg.layers, cfg.heads, cfg.kv_heads, cfg.intermediate) == \
        ("my-llama", 1024, 256, 2, 4, 2, 512)
    assert cfg.rope_scaling == {"factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                "original_max_position_embeddings": 256}
    assert cfg.bos_id == 1000 and cfg.eos_ids == (1001,) and cfg.rope_theta == 500000.0
    assert is_decoder(d) and not is_encoder(d)
    c = json.load(open(os.path.join(d, "config.json")))
    c["rope_scaling"] = {"rope_type": "yarn", "factor": 4.0}
    json.dump(c, open(os.path.join(d, "config.json"), "w"))
    with pytest.raises(ValueError):
        decoder_config(d)


def teacher_forced_agreement(hf, prompts, outs, tie_tol=0.02):
    """Fraction of generated tokens equal to the HF fp32 argmax on the generated prefix; every other
    token must be a near-tie of the HF logits (bf16 vs fp32): within ``tie_tol`` of the row's max
    |logit|."""
    exact = total = 0
    for p, t in zip(prompts, outs):
        seq = p + t[:-1]
        with torch.no_grad():
            lg = hf(torch.tensor([seq])).logits[0, len(p) - 1:].float()
        for j, tok in enumerate(t):
            total += 1
            best = int(lg[j].argmax())
            if tok == best:
                exact += 1
                continue
            gap = float(lg[j, best] - lg[j, tok])
            assert gap <= tie_tol * float(lg[j].abs().max()), (j, tok, best, gap)
    return exact / total


@pytest.mark.parametrize("tie", [False, True])
def test_llm_engine_runs_a_saved_hf_llama(tmp_path, bpe_dir, tie):
    """tie: Llama-3.2-style tied input / output embeddings (no lm_head tensor in the checkpoint)."""
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine, SamplingParams

    hf, d = _llama_dir(str(tmp_path), bpe_dir, rope_scaling=LLAMA3_SCALING, tie=tie)
    from django_assistant_bot_amd.models.configs import decoder_config

    assert decoder_config(d).tie_embeddings == tie
    eng = LLMEngine(d, device="cpu", max_batch=4, block_size=16, num_blocks=64, use_graphs=False)
    assert eng.tokenizer.byte_exact  # the directory's tokenizer.json, not the hash fallback
    prompts = [eng.tokenizer.encode(t) for t in ("the quick brown fox", "jumps over the lazy dog again")]
    sp = SamplingParams(max_new_tokens=10, do_sample=False, temperature=0.0, ignore_eos=True)
    outs = [o.token_ids for o in eng.generate(prompts, sp)]
    assert teacher_forced_agreement(hf, prompts, outs) >= 0.9


def test_embedding_engine_runs_a_saved_hf_bert(tmp_path):
    from django_assistant_bot_amd.engine.embedding_engine import EmbeddingEngine
    from django_assistant_bot_amd.models.configs import encoder_config, is_encoder

    torch.manual_seed(0)
    bc = transformers.BertConfig(vocab_size=2048, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                                 intermediate_size=256, max_position_embeddings=128)
    hf = transformers.BertModel(bc, add_pooling_layer=False).eval()
    d = str(tmp_path / "my-bert")
    hf.save_pretrained(d, safe_serialization=True)
    cfg = encoder_config(d)
    assert (cfg.hidden, cfg.layers, cfg.heads, cfg.intermediate, cfg.max_position) == (128, 2, 2, 256, 128)
    assert is_encoder(d)
    eng = EmbeddingEngine(d, device="cpu")
    ids = [[101, 5, 6, 7, 102], [101] + list(range(300, 340)) + [102]]
    import numpy as np

    flat = np.concatenate([np.asarray(s) for s in ids])
    offs = np.cumsum([0] + [len(s) for s in ids])
    ours = eng.embed_tokens(flat, offs)
    for i, s in enumerate(ids):
        with torch.no_grad():
            ref = hf(input_ids=torch.tensor([s])).last_hidden_state.mean(dim=1)[0]
        assert torch.allclose(ours[i].float(), ref, atol=5e-2), (ours[i] - ref).abs().max()


@pytest.mark.gpu
@pytest.mark.parametrize("tie", [False, True])
def test_llm_engine_runs_a_saved_hf_llama_on_gpu(tmp_path, bpe_dir, tie):
    """The GPU path at D = 128 (flash_d128 prefill with RoPE on load, the paged decode attention,
    fragment-layout stream GEMMs, HIP-graph decode) against HF fp32 with Llama-3 RoPE scaling."""
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine, SamplingParams

    hf, d = _llama_dir(str(tmp_path), bpe_dir, rope_scaling=LLAMA3_SCALING, hidden=512, heads=4, kv_heads=2, tie=tie)
    eng = LLMEngine(d, device="cuda", max_batch=8, block_size=64, num_blocks=64)
    assert eng.cfg.head_dim == 128 and eng.model.frag
    texts = ["the quick brown fox", "jumps over the lazy dog again and again", "a" * 300]
    prompts = [eng.tokenizer.encode(t) for t in texts]
    sp = SamplingParams(max_new_tokens=16, do_sample=False, temperature=0.0, ignore_eos=True)
    outs = [o.token_ids for o in eng.generate(prompts, sp)]
    assert eng.stats["graph_replays"] > 0
    # bf16 weights and activations against fp32 HF: one of the 48 tokens (tie=True) is HF's runner-up
    # at 2.02 % of the row's max |logit| when the 354-token prefill runs its GEMMs on gemm_mid, exact
    # on the 128 x 128 kernel.  Both kernels are equally accurate at these shapes (1 bf16 ulp on
    # 0.01-0.06 % of the elements against the fp32 reference, every epilogue:
    # benchmarks/gemm_mid_err_probe.py); a different rounding order flips that near-tie.
    assert teacher_forced_agreement(hf, prompts, outs, tie_tol=0.03) >= 0.85


LLAMA3_TEMPLATE = (
    "{{ bos_token }}{% for m in messages %}<|start_header_id|>{{ m['role'] }}<|end_header_id|>\n\n"
    "{{ m['content'] | trim }}<|eot_id|>{% endfor %}"
    "{% if add_generation_prompt %}<|start_header_id|>assistant<|end_header_id|>\n\n{% endif %}")


def test_chat_template_opt_in(tmp_path, bpe_dir):
    """ENGINE_CHAT_TEMPLATE: the provider renders messages with the checkpoint's chat template
    (tokenizer_config.json) instead of the reference's "role: content" lines; off by default."""
    import asyncio

    from assistant.ai.providers.transformers import TransformersProvider, render_prompt
    from assistant.conf import configure, reset
    from django_assistant_bot_amd.engine import serving

    _, d = _llama_dir(str(tmp_path), bpe_dir)
    json.dump({"chat_template": LLAMA3_TEMPLATE, "bos_token": "<|bos|>", "eos_token": {"content": "<|eos|>"}},
              open(os.path.join(d, "tokenizer_config.json"), "w"))
    p = TransformersProvider(d, device="cpu", max_batch=2, block_size=16, num_blocks=32, use_graphs=False)
    tok = p._tokenizer
    assert tok.has_chat_template
    msgs = [{"role": "system", "content": "be brief"}, {"role": "user", "content": "hi there "}]
    text = tok.render_chat(msgs)
    assert text == ("<|bos|><|start_header_id|>system<|end_header_id|>\n\nbe brief<|eot_id|>"
                    "<|start_header_id|>user<|end_header_id|>\n\nhi there<|eot_id|>"
                    "<|start_header_id|>assistant<|end_header_id|>\n\n")
    seen = []
    orig = p._worker.generate

    async def spy(ids, params):
        seen.append(list(ids))
        return await orig(ids, params)

    p._worker.generate = spy
    try:
        asyncio.run(p.get_response(msgs, max_tokens=4))
        configure(ENGINE_CHAT_TEMPLATE="true")
        asyncio.run(p.get_response(msgs, max_tokens=4))
    finally:
        reset("ENGINE_CHAT_TEMPLATE")
        with serving._lock:
            serving._llm.pop(d.lower(), None)
    assert seen[0] == tok.encode(render_prompt(msgs), add_special=True)
    assert seen[1] == tok.encode(text, add_special=False)
    # the sandbox refuses Python internals in a template
    from jinja2.exceptions import SecurityError

    tok._chat, tok._chat_fn = {"template": "{{ messages.__class__.__mro__ }}"}, None
    with pytest.raises(SecurityError):
        tok.render_chat(msgs)
