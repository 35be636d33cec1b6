"""Plain-PyTorch fp32 reference implementations of every native op.

They define the semantics the gfx950 kernels must match (tests compare kernel output against these)
and they are what runs when the engine is driven with CPU tensors (unit tests, the CPU plumbing
config of BASELINE.json).  Inputs/outputs use the same dtypes and layouts as the kernels.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

EPI_NONE, EPI_GELU, EPI_SWIGLU, EPI_SCORES = 0, 1, 2, 3
EPI_SWIGLU8 = 4  # SwiGLU over 8-row [gate | up] groups (decode copies of whole-chip stream_gemm tilings)


def rmsnorm(x, w, eps, residual=None):
    xf = x.float()
    res_out = None
    if residual is not None:
        xf = (xf + residual.float()).to(x.dtype).float()
        res_out = xf.to(x.dtype)
    inv = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * inv * w.float()).to(x.dtype), res_out


def layernorm(x, gamma, beta, eps, residual=None):
    xf = x.float()
    if residual is not None:
        xf = xf + residual.float()
    return F.layer_norm(xf, (x.shape[-1],), gamma.float(), beta.float(), eps).to(x.dtype)


def bert_embed(ids, pos_ids, type_ids, word, pos, typ, gamma, beta, eps):
    t = type_ids.long() if type_ids is not None else torch.zeros_like(ids, dtype=torch.long)
    e = word[ids.long()].float() + pos[pos_ids.long()].float() + typ[t].float()
    return F.layer_norm(e, (e.shape[-1],), gamma.float(), beta.float(), eps).to(word.dtype)


def embed_gather(ids, table):
    return table[ids.long()]


def mean_pool(hidden, cu_seqlens, normalize):
    cu = cu_seqlens.tolist()
    outs = []
    for i in range(len(cu) - 1):
        seg = hidden[cu[i]:cu[i + 1]].float()
        m = seg.mean(0) if seg.shape[0] else torch.zeros(hidden.shape[-1], device=hidden.device)
        outs.append(m)
    out = torch.stack(outs) if outs else hidden.new_zeros((0, hidden.shape[-1]), dtype=torch.float32)
    if normalize:
        out = F.normalize(out, dim=-1)
    return out


def gelu(x, bias=None):
    xf = x.float()
    if bias is not None:
        xf = xf + bias.float()
    return F.gelu(xf, approximate="none").to(x.dtype)


def silu_mul(x):
    F_ = x.shape[-1] // 2
    xf = x.float()
    return (F.silu(xf[..., :F_]) * xf[..., F_:]).to(x.dtype)


def rope_kv_write(qkv, positions, cos_sin, k_cache, v_cache, slots, Hq, Hkv, D, block_size):
    """Returns rotated q [T, Hq, D]; rotates k and writes k/v into the paged caches in place."""
    T = qkv.shape[0]
    x = qkv[:, : (Hq + 2 * Hkv) * D].float().view(T, Hq + 2 * Hkv, D)
    cs = cos_sin[positions.long()]  # [T, D/2, 2]
    cos, sin = cs[..., 0].unsqueeze(1), cs[..., 1].unsqueeze(1)
    half = D // 2
    qk = x[:, : Hq + Hkv]
    x1, x2 = qk[..., :half], qk[..., half:]
    rot = torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)
    q = rot[:, :Hq].to(qkv.dtype)
    k = rot[:, Hq:].to(qkv.dtype)
    v = x[:, Hq + Hkv:].to(qkv.dtype)
    for t in range(T):
        s = int(slots[t])
        if s < 0:
            continue
        blk, off = divmod(s, block_size)
        k_cache[blk, :, off] = k[t]
        v_cache[blk, :, off] = v[t]
    return q.contiguous()


def rope_q(q, positions, cos_sin):
    """Rotate-half RoPE of q [T, Hq, D] at ``positions`` (what rope_kv_write returns as q)."""
    D = q.shape[-1]
    half = D // 2
    cs = cos_sin[positions.long()]
    cos, sin = cs[..., 0].unsqueeze(1), cs[..., 1].unsqueeze(1)
    x = q.float()
    x1, x2 = x[..., :half], x[..., half:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(q.dtype)


def _attend(q, k, v, scale, causal, q_offset):
    # q [Sq, H, D], k/v [Sk, Hkv, D] -> [Sq, H, D] (fp32 math)
    H, Hkv = q.shape[1], k.shape[1]
    rep = H // Hkv
    kf = k.float().repeat_interleave(rep, dim=1)
    vf = v.float().repeat_interleave(rep, dim=1)
    s = torch.einsum("qhd,khd->hqk", q.float(), kf) * scale
    if causal:
        Sq, Sk = q.shape[0], k.shape[0]
        qpos = torch.arange(Sq, device=q.device)[:, None] + q_offset
        kpos = torch.arange(Sk, device=q.device)[None, :]
        s = s.masked_fill((kpos > qpos)[None], float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.einsum("hqk,khd->qhd", p, vf)


def flash_attention_packed(q, k, v, cu_q, cu_k, causal, scale):
    """q [Tq, Hq, D], k/v [Tk, Hkv, D] packed by cu_seqlens -> [Tq, Hq, D] (q dtype)."""
    out = torch.empty(q.shape, dtype=q.dtype, device=q.device)
    cq, ck = cu_q.tolist(), cu_k.tolist()
    for b in range(len(cq) - 1):
        qs, ks = q[cq[b]:cq[b + 1]], k[ck[b]:ck[b + 1]]
        vs = v[ck[b]:ck[b + 1]]
        off = ks.shape[0] - qs.shape[0]
        out[cq[b]:cq[b + 1]] = _attend(qs, ks, vs, scale, causal, off).to(q.dtype)
    return out


def gather_paged(cache, block_table, n):
    """cache [num_blocks, Hkv, bs, D] -> the first n tokens of a sequence as [n, Hkv, D]."""
    bs = cache.shape[2]
    nb = (n + bs - 1) // bs
    blocks = cache[block_table[:nb].long()]  # [nb, Hkv, bs, D]
    return blocks.permute(0, 2, 1, 3).reshape(nb * bs, cache.shape[1], cache.shape[3])[:n]


def flash_attention_paged(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, causal, scale):
    out = torch.empty(q.shape, dtype=q.dtype, device=q.device)
    cq = cu_q.tolist()
    for b in range(len(cq) - 1):
        n = int(ctx_lens[b])
        ks = gather_paged(k_cache, block_tables[b], n)
        vs = gather_paged(v_cache, block_tables[b], n)
        qs = q[cq[b]:cq[b + 1]]
        out[cq[b]:cq[b + 1]] = _attend(qs, ks, vs, scale, causal, n - qs.shape[0]).to(q.dtype)
    return out


def paged_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale):
    """q [B, Hq, D] one token per sequence -> [B, Hq, D]."""
    out = torch.empty(q.shape, dtype=q.dtype, device=q.device)
    for b in range(q.shape[0]):
        n = int(ctx_lens[b])
        ks = gather_paged(k_cache, block_tables[b], n)
        vs = gather_paged(v_cache, block_tables[b], n)
        out[b] = _attend(q[b:b + 1], ks, vs, scale, False, 0)[0].to(q.dtype)
    return out


def gemm_bt(A, B, bias=None, residual=None, epilogue=EPI_NONE, out_f32=False, row_group=None, q_group=None,
            allow=None):
    c = A.float() @ B.float().t()
    if epilogue == EPI_SCORES:
        ok = torch.ones_like(c, dtype=torch.bool)
        if row_group is not None:
            rg = row_group.long()[None, :]
            ok &= rg >= 0
            if q_group is not None:
                qg = q_group.long()[:, None]
                ok &= (qg < 0) | (rg == qg)
        if allow is not None:
            n = c.shape[1]
            idx = torch.arange(n, device=c.device)
            bits = (allow[:, idx // 32].long() >> (idx % 32)) & 1
            ok &= bits.bool()
        c = c.masked_fill(~ok, float("-inf"))
        return c if out_f32 else c.to(A.dtype)
    if bias is not None:
        c = c + bias.float()
    if epilogue == EPI_GELU:
        c = F.gelu(c)
    elif epilogue in (EPI_SWIGLU, EPI_SWIGLU8):
        N, hg = c.shape[1], 16 if epilogue == EPI_SWIGLU else 8
        c = c.view(c.shape[0], N // (2 * hg), 2, hg)
        c = (F.silu(c[:, :, 0]) * c[:, :, 1]).reshape(c.shape[0], N // 2)
    if residual is not None:
        # a bf16 output is the rounded projection plus the residual, rounded again (HF's
        # `hidden + dense(x)` in bf16)
        c = (c if out_f32 else c.to(A.dtype).float()) + residual.float()
    return c if out_f32 else c.to(A.dtype)


def sample_hf(logits, temperature, top_k, top_p, generator=None):
    """HF generate() logits-warper semantics: temperature -> top-k -> top-p -> multinomial."""
    out = []
    for r in range(logits.shape[0]):
        x = logits[r].float()
        t = float(temperature[r])
        if t <= 0:
            out.append(int(torch.argmax(x)))
            continue
        x = x / t
        k = int(top_k[r])
        if 0 < k < x.numel():
            kth = torch.topk(x, k).values[-1]
            x = x.masked_fill(x < kth, float("-inf"))
        p = float(top_p[r])
        if p < 1.0:
            sl, si = torch.sort(x, descending=False)
            cum = torch.softmax(sl, -1).cumsum(-1)
            remove = cum <= (1 - p)
            remove[-1] = False
            x = x.masked_fill(torch.zeros_like(remove).scatter(0, si, remove), float("-inf"))
        probs = torch.softmax(x, -1)
        out.append(int(torch.multinomial(probs, 1, generator=generator)))
    return torch.tensor(out, dtype=torch.int32, device=logits.device)


def topk_rows(scores, k):
    v, i = torch.topk(scores.float(), k, dim=-1, largest=True, sorted=True)
    return v, i.to(torch.int32)


def rope_cos_sin(inv_freq: torch.Tensor, max_pos: int) -> torch.Tensor:
    t = torch.arange(max_pos, dtype=torch.float32)
    f = torch.outer(t, inv_freq.float())
    return torch.stack([f.cos(), f.sin()], dim=-1).contiguous()  # [max_pos, D/2, 2]


def llama3_inv_freq(D, theta, scaling=None):
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, dtype=torch.float32) / D))
    if not scaling:
        return inv
    factor = scaling.get("factor", 8.0)
    lo = scaling.get("low_freq_factor", 1.0)
    hi = scaling.get("high_freq_factor", 4.0)
    orig = scaling.get("original_max_position_embeddings", 8192)
    lo_wl, hi_wl = orig / lo, orig / hi
    wl = 2 * math.pi / inv
    out = torch.where(wl > lo_wl, inv / factor, inv)
    smooth = (orig / wl - lo) / (hi - lo)
    mid = (1 - smooth) * out / factor + smooth * out
    is_mid = (wl >= hi_wl) & (wl <= lo_wl)
    return torch.where(is_mid, mid, out)
