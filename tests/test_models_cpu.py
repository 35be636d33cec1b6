"""Model semantics on CPU (reference ops): parity with HF transformers BertModel / LlamaForCausalLM
built from the same weights -- the reference runs exactly those HF classes (ai/embedders/transformers.py,
ai/providers/transformers.py)."""
import math

import pytest
import torch

from django_assistant_bot_amd.models import (AttnMeta, BertEncoder, KVCache, LlamaModel, decoder_config,
                                             encoder_config, pack_sequences, random_decoder_weights,
                                             random_encoder_weights, shard_decoder_weights)

transformers = pytest.importorskip("transformers")


def test_bert_matches_hf_mean_pool():
    cfg = encoder_config("tiny-bert")
    w = {k: v.float() for k, v in random_encoder_weights(cfg, dtype=torch.float32, seed=3).items()}
    hf_cfg = transformers.BertConfig(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden, num_hidden_layers=cfg.layers,
                                     num_attention_heads=cfg.heads, intermediate_size=cfg.intermediate,
                                     max_position_embeddings=cfg.max_position, layer_norm_eps=cfg.eps,
                                     hidden_act="gelu", attn_implementation="eager")
    hf = transformers.BertModel(hf_cfg, add_pooling_layer=False).eval()
    H = cfg.hidden
    sd = {"embeddings.word_embeddings.weight": w["word_emb"], "embeddings.position_embeddings.weight": w["pos_emb"],
          "embeddings.token_type_embeddings.weight": w["type_emb"], "embeddings.LayerNorm.weight": w["emb_ln_g"],
          "embeddings.LayerNorm.bias": w["emb_ln_b"]}
    for i in range(cfg.layers):
        p = f"encoder.layer.{i}."
        for j, n in enumerate(("query", "key", "value")):
            sd[p + f"attention.self.{n}.weight"] = w[f"l{i}.qkv_w"][j * H:(j + 1) * H]
            sd[p + f"attention.self.{n}.bias"] = w[f"l{i}.qkv_b"][j * H:(j + 1) * H]
        sd[p + "attention.output.dense.weight"] = w[f"l{i}.o_w"]
        sd[p + "attention.output.dense.bias"] = w[f"l{i}.o_b"]
        sd[p + "attention.output.LayerNorm.weight"] = w[f"l{i}.ln1_g"]
        sd[p + "attention.output.LayerNorm.bias"] = w[f"l{i}.ln1_b"]
        sd[p + "intermediate.dense.weight"] = w[f"l{i}.i_w"]
        sd[p + "intermediate.dense.bias"] = w[f"l{i}.i_b"]
        sd[p + "output.dense.weight"] = w[f"l{i}.d_w"]
        sd[p + "output.dense.bias"] = w[f"l{i}.d_b"]
        sd[p + "output.LayerNorm.weight"] = w[f"l{i}.ln2_g"]
        sd[p + "output.LayerNorm.bias"] = w[f"l{i}.ln2_b"]
    missing, unexpected = hf.load_state_dict(sd, strict=False)
    assert not unexpected and all("position_ids" in m or "token_type" in m for m in missing)
    enc = BertEncoder(cfg, w, "cpu")
    seqs = [[101, 5, 6, 7, 102], [101, 900, 102], [101] + list(range(10, 40)) + [102]]
    ids, pos, cu, mx = pack_sequences(seqs, "cpu")
    ours = enc.encode(ids, pos, cu, mx)
    for i, s in enumerate(seqs):
        with torch.no_grad():
            ref = hf(input_ids=torch.tensor([s])).last_hidden_state.mean(dim=1)[0]  # the reference's pooling
        assert torch.allclose(ours[i], ref, atol=2e-4), (ours[i] - ref).abs().max()


def _llama_pair(seed=1):
    cfg = decoder_config("tiny-llama")
    full = {k: v.float() for k, v in random_decoder_weights(cfg, dtype=torch.float32, seed=seed).items()}
    return cfg, full


def _hf_llama(cfg, full):
    hc = transformers.LlamaConfig(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden, num_hidden_layers=cfg.layers,
                                  num_attention_heads=cfg.heads, num_key_value_heads=cfg.kv_heads,
                                  intermediate_size=cfg.intermediate, rms_norm_eps=cfg.eps, rope_theta=cfg.rope_theta,
                                  max_position_embeddings=cfg.max_position, tie_word_embeddings=False,
                                  attn_implementation="eager")
    hf = transformers.LlamaForCausalLM(hc).eval()
    D, F = cfg.head_dim, cfg.intermediate
    sd = {"model.embed_tokens.weight": full["embed"], "model.norm.weight": full["final_norm"],
          "lm_head.weight": full["lm_head"]}
    qn, kn = cfg.heads * D, cfg.kv_heads * D
    for i in range(cfg.layers):
        p = f"model.layers.{i}."
        qkv = full[f"l{i}.qkv_w"]
        sd[p + "self_attn.q_proj.weight"] = qkv[:qn]
        sd[p + "self_attn.k_proj.weight"] = qkv[qn:qn + kn]
        sd[p + "self_attn.v_proj.weight"] = qkv[qn + kn:]
        sd[p + "self_attn.o_proj.weight"] = full[f"l{i}.o_w"]
        sd[p + "mlp.gate_proj.weight"] = full[f"l{i}.gate_up_w"][:F]
        sd[p + "mlp.up_proj.weight"] = full[f"l{i}.gate_up_w"][F:]
        sd[p + "mlp.down_proj.weight"] = full[f"l{i}.down_w"]
        sd[p + "input_layernorm.weight"] = full[f"l{i}.attn_norm"]
        sd[p + "post_attention_layernorm.weight"] = full[f"l{i}.mlp_norm"]
    hf.load_state_dict(sd, strict=True)
    return hf


def _prefill(model, cfg, ids, bs=64, nb=8):
    kv = KVCache(cfg.layers, nb, cfg.kv_heads // model.tp_size, bs, cfg.head_dim, "cpu", dtype=torch.float32)
    T = len(ids)
    bt = torch.arange(nb, dtype=torch.int32)[None]
    meta = AttnMeta(decode=False, positions=torch.arange(T, dtype=torch.int32), slots=torch.arange(T),
                    block_tables=bt, ctx_lens=torch.tensor([T], dtype=torch.int32),
                    cu_q=torch.tensor([0, T], dtype=torch.int32), max_q=T)
    return model.forward(torch.tensor(ids, dtype=torch.int32), meta, kv), kv


def test_llama_prefill_matches_hf():
    cfg, full = _llama_pair()
    hf = _hf_llama(cfg, full)
    model = LlamaModel(cfg, full, "cpu")
    ids = [5, 17, 300, 42, 999, 7, 1, 64, 65, 66]
    h, _ = _prefill(model, cfg, ids)
    ours = model.logits(h)
    with torch.no_grad():
        ref = hf(torch.tensor([ids])).logits[0]
    assert torch.allclose(ours, ref, atol=1e-3, rtol=1e-3), (ours - ref).abs().max()


def test_llama_decode_consistent_with_prefill():
    cfg, full = _llama_pair(2)
    model = LlamaModel(cfg, full, "cpu")
    ids = list(range(3, 3 + 70))  # crosses a 64-token block
    h_full, _ = _prefill(model, cfg, ids)
    h_pre, kv = _prefill(model, cfg, ids[:-1])
    T = len(ids)
    meta = AttnMeta(decode=True, positions=torch.tensor([T - 1], dtype=torch.int32), slots=torch.tensor([T - 1]),
                    block_tables=torch.arange(8, dtype=torch.int32)[None], ctx_lens=torch.tensor([T], dtype=torch.int32))
    h_dec = model.forward(torch.tensor([ids[-1]], dtype=torch.int32), meta, kv)
    assert torch.allclose(h_dec[0], h_full[-1], atol=1e-4)


def test_tensor_parallel_shards_reconstruct_full_model():
    """Sum of per-shard row-parallel outputs == unsharded projection (Megatron split used by TP)."""
    cfg, full = _llama_pair(4)
    tp = 2
    shards = [shard_decoder_weights(full, cfg, r, tp) for r in range(tp)]
    x = torch.randn(3, cfg.hidden)
    D, F = cfg.head_dim, cfg.intermediate
    # attention output projection: concatenated head outputs x_heads @ o_w^T == sum over shards
    heads = torch.randn(3, cfg.heads * D)
    ref = heads @ full["l0.o_w"].t()
    hq = cfg.heads // tp
    got = sum(heads[:, r * hq * D:(r + 1) * hq * D] @ shards[r]["l0.o_w"].t() for r in range(tp))
    assert torch.allclose(got, ref, atol=1e-5)
    # MLP: silu(gate) * up, down-projected, summed over shards
    gu = x @ full["l0.gate_up_w"].t()
    ref = (torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]) @ full["l0.down_w"].t()
    got = 0
    for r in range(tp):
        g = x @ shards[r]["l0.gate_up_w"].t()
        f = F // tp
        got = got + (torch.nn.functional.silu(g[:, :f]) * g[:, f:]) @ shards[r]["l0.down_w"].t()
    assert torch.allclose(got, ref, atol=1e-4)
    assert math.isclose(sum(s["l0.qkv_w"].numel() for s in shards), full["l0.qkv_w"].numel())


def test_llama_interleaved_mlp_layout_matches():
    """8-row interleaved gate|up weights (the engine's fused-SwiGLU layout) give the same model."""
    from django_assistant_bot_amd.models.weights import _gate_up

    cfg, full = _llama_pair(3)
    inter = dict(full)
    F = cfg.intermediate
    for i in range(cfg.layers):
        gu = full[f"l{i}.gate_up_w"]
        inter[f"l{i}.gate_up_w"] = _gate_up(gu[:F], gu[F:], True)
    ids = list(range(5, 40))
    h_a, _ = _prefill(LlamaModel(cfg, full, "cpu"), cfg, ids)
    h_b, _ = _prefill(LlamaModel(cfg, inter, "cpu", interleaved_mlp=True), cfg, ids)
    assert torch.allclose(h_a, h_b, atol=1e-5)


def test_random_tp_shards_replicate_embedding_and_lm_head():
    cfg = decoder_config("tiny-llama")
    a = random_decoder_weights(cfg, dtype=torch.float32, seed=4, tp_rank=0, tp_size=2)
    b = random_decoder_weights(cfg, dtype=torch.float32, seed=4, tp_rank=1, tp_size=2)
    assert torch.equal(a["embed"], b["embed"]) and torch.equal(a["lm_head"], b["lm_head"])
    assert not torch.equal(a["l0.qkv_w"], b["l0.qkv_w"])
    full = random_decoder_weights(cfg, dtype=torch.float32, seed=4)
    assert torch.equal(shard_decoder_weights(full, cfg, 1, 2)["lm_head"], full["lm_head"])


def test_gate_up_regroup_and_swiglu8_reference():
    """The decode copy of gate_up is regrouped from 16-row to 8-row [gate | up] pairs (any 16-row
    multiple then tiles it); the EPI_SWIGLU8 reference equals SiLU(gate) * up of the plain layout."""
    from django_assistant_bot_amd import ops
    from django_assistant_bot_amd.ops import reference as ref

    F, H = 112, 64
    g, u, x = torch.randn(F, H), torch.randn(F, H), torch.randn(5, H)
    w16 = ops.interleave_gate_up(g, u)
    w8 = ops.regroup_gate_up(w16, 16, 8)
    assert torch.equal(w8, ops.interleave_gate_up(g, u, 8))
    exp = torch.nn.functional.silu(x @ g.t()) * (x @ u.t())
    got8 = ref.gemm_bt(x, w8, epilogue=ops.EPI_SWIGLU8, out_f32=True)
    got16 = ref.gemm_bt(x, w16, epilogue=ops.EPI_SWIGLU, out_f32=True)
    torch.testing.assert_close(got8, exp, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(got16, exp, atol=1e-4, rtol=1e-4)


def _hf_checkpoint(tmp_path, cfg, full):
    """The state in HF Llama tensor names, split over two safetensors files."""
    from safetensors.torch import save_file

    H, D, F = cfg.hidden, cfg.head_dim, cfg.intermediate
    hf = {"model.embed_tokens.weight": full["embed"], "model.norm.weight": full["final_norm"]}
    if "lm_head" in full:
        hf["lm_head.weight"] = full["lm_head"]
    for i in range(cfg.layers):
        p = f"model.layers.{i}."
        qkv = full[f"l{i}.qkv_w"]
        hf[p + "self_attn.q_proj.weight"] = qkv[: cfg.heads * D]
        hf[p + "self_attn.k_proj.weight"] = qkv[cfg.heads * D:(cfg.heads + cfg.kv_heads) * D]
        hf[p + "self_attn.v_proj.weight"] = qkv[(cfg.heads + cfg.kv_heads) * D:]
        hf[p + "self_attn.o_proj.weight"] = full[f"l{i}.o_w"]
        hf[p + "mlp.gate_proj.weight"] = full[f"l{i}.gate_up_w"][:F]
        hf[p + "mlp.up_proj.weight"] = full[f"l{i}.gate_up_w"][F:]
        hf[p + "mlp.down_proj.weight"] = full[f"l{i}.down_w"]
        hf[p + "input_layernorm.weight"] = full[f"l{i}.attn_norm"]
        hf[p + "post_attention_layernorm.weight"] = full[f"l{i}.mlp_norm"]
    keys = sorted(hf)
    half = len(keys) // 2
    save_file({k: hf[k].contiguous() for k in keys[:half]}, str(tmp_path / "model-00001-of-00002.safetensors"))
    save_file({k: hf[k].contiguous() for k in keys[half:]}, str(tmp_path / "model-00002-of-00002.safetensors"))
    return hf


def test_tp_checkpoint_load_reads_only_the_rank_slices(tmp_path):
    """VERDICT r2 "next" #4: each TP rank materialises ~1/tp of the projection bytes of a multi-file
    checkpoint (safetensors get_slice), and its shard equals shard_decoder_weights(full state)."""
    from django_assistant_bot_amd.models.weights import SafetensorsDir, load_decoder_checkpoint

    cfg = decoder_config("tiny-llama-70b-layout")
    full = random_decoder_weights(cfg, dtype=torch.float32, seed=11)
    hf = _hf_checkpoint(tmp_path, cfg, full)
    proj = sum(v.numel() * 4 for k, v in hf.items() if "_proj" in k)
    repl = sum(v.numel() * 4 for k, v in hf.items() if "_proj" not in k)
    for tp in (2, 4, 8):
        for r in (0, tp - 1):
            st = SafetensorsDir(str(tmp_path))
            got = load_decoder_checkpoint(str(tmp_path), cfg, dtype=torch.float32, tp_rank=r, tp_size=tp,
                                          interleave_mlp=True, reader=st)
            want = shard_decoder_weights(full, cfg, r, tp, interleave_mlp=True)
            assert set(got) == set(want)
            for k in want:
                assert torch.equal(got[k], want[k]), (tp, r, k)
            assert st.bytes_read <= repl + proj / tp * 1.001, (tp, st.bytes_read, repl, proj)




@pytest.mark.parametrize("group", [1, 7, 8])
def test_grouped_fragment_layout_round_trip_and_addressing(group):
    """``shuffle_weights(w, G)``: a permutation of the rows' 1-KB fragments -- fragment (block b, k
    chunk c) of the plain layout sits at 1-KB slot ((b / G) K/32 + c) G + b % G, the address the
    kernels compute (stream_gemm.hip ``wblk``, gemm_mid / gemm256 / gemm.hip ``bgrp``); the inverse
    restores the matrix and the CPU gemm_bt fallback reads it with ``b_group``."""
    from django_assistant_bot_amd import ops
    N, K = 16 * group * 3, 128
    w = torch.randn(N, K).to(torch.bfloat16)
    plain, grp = ops.shuffle_weights(w).view(-1, 512), ops.shuffle_weights(w, group).view(-1, 512)
    nck = K // 32
    for b in range(N // 16):
        for c in range(nck):
            assert torch.equal(grp[((b // group) * nck + c) * group + b % group], plain[b * nck + c])
    assert torch.equal(ops.unshuffle_weights(ops.shuffle_weights(w, group), group), w)
    if group == 8:
        x = torch.randn(5, K).to(torch.bfloat16)
        assert torch.equal(ops.gemm_bt(x, ops.shuffle_weights(w, 8), shuffled=True, b_group=8),
                           ops.gemm_bt(x, w))
