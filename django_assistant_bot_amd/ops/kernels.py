"""Tensor-level wrappers of the gfx950 kernels.

Each function validates shapes / dtypes / devices on the host BEFORE launching (a hand-written
kernel that is fed a wrong shape faults the GPU), then enqueues on the current HIP stream, which
makes every op capturable into a HIP graph.  CPU tensors run ``ops.reference``.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import reference as ref
from ._lib import expect, expect_bf16_contig, native, ptr, same_device, stream

EPI_NONE, EPI_GELU, EPI_SWIGLU, EPI_SCORES = ref.EPI_NONE, ref.EPI_GELU, ref.EPI_SWIGLU, ref.EPI_SCORES
EPI_SWIGLU8 = ref.EPI_SWIGLU8


def _i32(t: torch.Tensor) -> None:
    if t.dtype != torch.int32 or not t.is_contiguous():
        raise TypeError("expected a contiguous int32 tensor")


# ----------------------------------------------------------------------------------------------
# normalisation / embeddings / pooling


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: torch.Tensor | None = None):
    """RMSNorm over the last dim; with ``residual`` the input is ``x + residual`` and the sum is
    also returned (fused residual stream).  Returns (out, residual_out).

    ``x`` may also be split-K slabs [S, rows, cols] (fp32, or bf16: ``slab_dtype``) of the producing
    projection (``stream_gemm(..., splits=S)``): they are summed in fp32 (and rounded to bf16) inside
    the kernel."""
    slabs = x.dim() == 3 and x.dtype in (torch.float32, torch.bfloat16)
    if not x.is_cuda:
        if slabs:
            x = x.float().sum(0).to(torch.bfloat16)
        return ref.rmsnorm(x, w, eps, residual)
    expect_bf16_contig(w, residual)
    same_device(x, w, residual)
    cols = x.shape[-1]
    expect(w.numel() == cols, "rmsnorm weight size mismatch")
    if slabs:
        expect(x.is_contiguous(), "slabs must be contiguous")
        S, rows = x.shape[0], x.shape[1]
        shape = (rows, cols)
    else:
        expect_bf16_contig(x)
        rows = x.numel() // cols
        shape = tuple(x.shape)
    expect(residual is None or tuple(residual.shape) == shape, "residual shape mismatch")
    out = torch.empty(shape, dtype=torch.bfloat16, device=x.device)
    res_out = torch.empty(shape, dtype=torch.bfloat16, device=x.device) if residual is not None else None
    if slabs:
        native().rmsnorm_slabs(ptr(out), ptr(res_out), ptr(x), S, rows * cols, ptr(residual), ptr(w), rows, cols,
                               float(eps), stream(x), int(x.dtype == torch.bfloat16))
    else:
        native().rmsnorm(ptr(out), ptr(res_out), ptr(x), ptr(residual), ptr(w), rows, cols, float(eps), stream(x))
    return out, res_out


def layernorm(x, gamma, beta, eps, residual=None):
    if not x.is_cuda:
        return ref.layernorm(x, gamma, beta, eps, residual)
    expect_bf16_contig(x, gamma, beta, residual)
    same_device(x, gamma, beta, residual)
    cols = x.shape[-1]
    rows = x.numel() // cols
    expect(gamma.numel() == cols and beta.numel() == cols, "layernorm affine size mismatch")
    expect(residual is None or residual.shape == x.shape, "residual shape mismatch")
    out = torch.empty_like(x)
    native().layernorm(ptr(out), ptr(x), ptr(residual), ptr(gamma), ptr(beta), rows, cols, float(eps), stream(x))
    return out


def bert_embed(ids, pos_ids, type_ids, word, pos, typ, gamma, beta, eps):
    if not ids.is_cuda:
        return ref.bert_embed(ids, pos_ids, type_ids, word, pos, typ, gamma, beta, eps)
    _i32(ids)
    _i32(pos_ids)
    if type_ids is not None:
        _i32(type_ids)
    expect_bf16_contig(word, pos, typ, gamma, beta)
    expect(ids.shape == pos_ids.shape, "ids / position ids mismatch")
    H = word.shape[1]
    out = torch.empty((ids.numel(), H), dtype=word.dtype, device=ids.device)
    native().bert_embed(ptr(out), ptr(ids), ptr(pos_ids), ptr(type_ids), ptr(word), ptr(pos), ptr(typ), ptr(gamma),
                        ptr(beta), ids.numel(), H, float(eps), stream(ids))
    return out


def embed_gather(ids, table):
    if not ids.is_cuda:
        return ref.embed_gather(ids, table)
    _i32(ids)
    expect_bf16_contig(table)
    out = torch.empty((ids.numel(), table.shape[1]), dtype=table.dtype, device=ids.device)
    native().embed_gather(ptr(out), ptr(ids), ptr(table), ids.numel(), table.shape[1], stream(ids))
    return out


def mean_pool(hidden, cu_seqlens, normalize=False, want_bf16=False):
    """Mean over each packed sequence (all tokens, as the reference).  Returns fp32 [B, H]
    (and a bf16 copy when ``want_bf16``)."""
    if not hidden.is_cuda:
        out = ref.mean_pool(hidden, cu_seqlens, normalize)
        return (out, out.to(torch.bfloat16)) if want_bf16 else out
    expect_bf16_contig(hidden)
    _i32(cu_seqlens)
    B = cu_seqlens.numel() - 1
    H = hidden.shape[1]
    expect(H <= 4096, "mean_pool supports hidden <= 4096")
    out = torch.empty((B, H), dtype=torch.float32, device=hidden.device)
    ob = torch.empty((B, H), dtype=torch.bfloat16, device=hidden.device) if want_bf16 else None
    native().mean_pool(ptr(out), ptr(ob), ptr(hidden), ptr(cu_seqlens), B, H, int(bool(normalize)), stream(hidden))
    return (out, ob) if want_bf16 else out


# ----------------------------------------------------------------------------------------------
# element-wise


def gelu(x, bias=None, out=None):
    if not x.is_cuda:
        return ref.gelu(x, bias)
    expect_bf16_contig(x, bias)
    cols = x.shape[-1]
    out = torch.empty_like(x) if out is None else out
    native().gelu(ptr(out), ptr(x), ptr(bias), x.numel() // cols, cols, stream(x))
    return out


def silu_mul(x, interleaved=False, group: int | None = None):
    """x [..., 2F] = [gate | up] -> silu(gate) * up  [..., F].  ``group`` (or ``interleaved`` = 16):
    x columns are ``group``-wide [gate | up] groups (the projection of ``interleave_gate_up``
    weights; 0 = stacked halves)."""
    group = (16 if interleaved else 0) if group is None else int(group)
    if not x.is_cuda:
        if group:
            F2 = x.shape[-1]
            v = x.reshape(*x.shape[:-1], F2 // (2 * group), 2, group)
            x = torch.cat([v[..., 0, :].reshape(*x.shape[:-1], F2 // 2), v[..., 1, :].reshape(*x.shape[:-1], F2 // 2)], -1)
        return ref.silu_mul(x)
    expect(group in (0, 16), "the GPU silu_mul takes stacked or 16-column groups (8-row groups: EPI_SWIGLU8)")
    expect_bf16_contig(x)
    F2 = x.shape[-1]
    rows = x.numel() // F2
    out = torch.empty((*x.shape[:-1], F2 // 2), dtype=x.dtype, device=x.device)
    native().silu_mul(ptr(out), ptr(x), rows, F2 // 2, stream(x), int(group == 16))
    return out


def rope_kv_write(qkv, positions, cos_sin, k_cache, v_cache, slots, Hq, Hkv, D, write_q=True):
    """Applies RoPE to the q/k heads of ``qkv`` [T, (Hq+2Hkv)*D]; writes k, v into the paged caches
    [num_blocks, Hkv, block_size, D] at ``slots`` (int64, <0 skipped); returns q [T, Hq, D].
    ``qkv`` may also be split-K slabs [S, T, (Hq+2Hkv)*D] (fp32 or bf16), summed inside the kernel.
    ``write_q=False`` (bf16 ``qkv``): k / v only, returns None (the prefill attention rotates q on
    load: ``flash_attention_paged(..., rope=...)``)."""
    block_size = k_cache.shape[2]
    slabs = qkv.dim() == 3 and qkv.dtype in (torch.float32, torch.bfloat16)
    if not qkv.is_cuda:
        if slabs:
            qkv = qkv.float().sum(0).to(torch.bfloat16)
        return ref.rope_kv_write(qkv, positions, cos_sin, k_cache, v_cache, slots, Hq, Hkv, D, block_size)
    expect_bf16_contig(k_cache, v_cache)
    _i32(positions)
    expect(slots.dtype == torch.int64 and slots.is_contiguous(), "slots must be contiguous int64")
    expect(cos_sin.dtype == torch.float32 and cos_sin.is_contiguous(), "cos_sin must be contiguous fp32")
    T = qkv.shape[-2]
    expect(qkv.shape[-1] == (Hq + 2 * Hkv) * D, "qkv width mismatch")
    expect(positions.numel() == T and slots.numel() == T, "positions / slots length mismatch")
    expect(tuple(k_cache.shape[1:]) == (Hkv, block_size, D) and k_cache.shape == v_cache.shape, "cache shape mismatch")
    expect(cos_sin.shape[1] == D // 2, "cos/sin table width mismatch")
    if not write_q:
        expect(not slabs, "write_q=False needs a bf16 qkv")
        expect_bf16_contig(qkv)
        native().rope_kv_write(ptr(qkv), qkv.stride(0), ptr(positions), ptr(cos_sin), 0, ptr(k_cache),
                               ptr(v_cache), ptr(slots), T, Hq, Hkv, D, block_size, stream(qkv))
        return None
    q = torch.empty((T, Hq, D), dtype=torch.bfloat16, device=qkv.device)
    if slabs:
        expect(qkv.is_contiguous(), "slabs must be contiguous")
        native().rope_kv_write(0, qkv.shape[-1], ptr(positions), ptr(cos_sin), ptr(q), ptr(k_cache), ptr(v_cache),
                               ptr(slots), T, Hq, Hkv, D, block_size, stream(qkv), ptr(qkv), qkv.shape[0],
                               T * qkv.shape[-1], int(qkv.dtype == torch.bfloat16))
    else:
        expect_bf16_contig(qkv)
        native().rope_kv_write(ptr(qkv), qkv.stride(0), ptr(positions), ptr(cos_sin), ptr(q), ptr(k_cache),
                               ptr(v_cache), ptr(slots), T, Hq, Hkv, D, block_size, stream(qkv))
    return q


# ----------------------------------------------------------------------------------------------
# attention


def _head_strides(t: torch.Tensor):
    # t viewed as [tokens, heads, D] with unit stride on D
    expect(t.stride(-1) == 1, "attention operands need unit stride on the head dim")
    return t.stride(0), t.stride(1)


def flash_attention_packed(q, k, v, cu_q, cu_k, max_seqlen_q, causal=False, scale=None, out=None):
    """Variable-length attention over packed sequences.  q [Tq, Hq, D], k/v [Tk, Hkv, D] may be
    strided views of a fused QKV buffer.  Returns [Tq, Hq, D] contiguous."""
    D = q.shape[-1]
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if not q.is_cuda:
        return ref.flash_attention_packed(q, k, v, cu_q, cu_k, causal, scale)
    _i32(cu_q)
    _i32(cu_k)
    expect(q.dtype == torch.bfloat16 and k.dtype == torch.bfloat16 and v.dtype == torch.bfloat16, "bf16 required")
    expect(D in (32, 64, 128), "head dim must be 32, 64 or 128")
    Hq, Hkv = q.shape[1], k.shape[1]
    expect(Hq % Hkv == 0, "GQA requires Hq % Hkv == 0")
    expect(k.stride() == v.stride(), "k and v must share strides")
    qst, qsh = _head_strides(q)
    kst, ksh = _head_strides(k)
    for s in (qst, qsh, kst, ksh):
        expect(s % 8 == 0, "attention strides must be multiples of 8 elements (16 B)")
    out = torch.empty((q.shape[0], Hq, D), dtype=q.dtype, device=q.device) if out is None else out
    B = cu_q.numel() - 1
    native().flash_attention(ptr(q), qst, qsh, ptr(k), ptr(v), kst, ksh, 0, 0, 0, 0, 0, ptr(out), out.stride(0),
                             out.stride(1), ptr(cu_q), ptr(cu_k), 0, B, int(max_seqlen_q), Hq, Hkv, D,
                             int(bool(causal)), 0, float(scale), stream(q))
    return out


def flash_rope_ok(D: int, block_size: int) -> bool:
    """Whether flash_attention_paged can rotate q itself (the 32x32 D = 128 kernel's Q prologue)."""
    return D == 128 and block_size % 64 == 0


def flash_attention_paged(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, max_seqlen_q, causal=True, scale=None,
                          out=None, rope=None):
    """Prefill attention: q [Tq, Hq, D] packed by cu_q, keys/values of each sequence are its first
    ctx_lens[b] tokens in the paged caches (the query chunk is the tail of that context).
    ``rope=(positions int32 [Tq], cos_sin [max_pos, D/2, 2] fp32)``: q is the un-rotated projection
    and RoPE is applied on load (``flash_rope_ok``)."""
    D = q.shape[-1]
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if not q.is_cuda:
        if rope is not None:
            pos, cs = rope
            T, Hq = q.shape[0], q.shape[1]
            q = ref.rope_q(q.reshape(T, Hq, D), pos, cs)
        return ref.flash_attention_paged(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, causal, scale)
    _i32(cu_q)
    _i32(ctx_lens)
    _i32(block_tables)
    expect_bf16_contig(k_cache, v_cache)
    expect(D in (32, 64, 128), "head dim must be 32, 64 or 128")
    Hq, Hkv, bs = q.shape[1], k_cache.shape[1], k_cache.shape[2]
    qst, qsh = _head_strides(q)
    out = torch.empty((q.shape[0], Hq, D), dtype=q.dtype, device=q.device) if out is None else out
    B = cu_q.numel() - 1
    expect(block_tables.shape[0] >= B and ctx_lens.numel() >= B, "block table / ctx_lens rows < batch")
    if rope is not None:
        pos, cs = rope
        _i32(pos)
        expect(flash_rope_ok(D, bs) and cs.dtype == torch.float32 and cs.is_contiguous() and pos.numel() == q.shape[0],
               "q RoPE in the attention needs D 128, block size % 64, fp32 cos/sin and one position per query")
        native().flash_attention_rope(ptr(q), qst, qsh, ptr(k_cache), ptr(v_cache), ptr(block_tables),
                                      block_tables.shape[1], bs, ptr(out), out.stride(0), out.stride(1), ptr(cu_q),
                                      ptr(ctx_lens), B, int(max_seqlen_q), Hq, Hkv, D, int(bool(causal)),
                                      float(scale), ptr(pos), ptr(cs), stream(q))
        return out
    native().flash_attention(ptr(q), qst, qsh, 0, 0, 0, 0, ptr(k_cache), ptr(v_cache), ptr(block_tables),
                             block_tables.shape[1], bs, ptr(out), out.stride(0), out.stride(1), ptr(cu_q), 0,
                             ptr(ctx_lens), B, int(max_seqlen_q), Hq, Hkv, D, int(bool(causal)), 1, float(scale),
                             stream(q))
    return out


class DecodeWorkspace:
    """Partition buffers of the split-K paged decode; allocated once (graph-capture safe)."""

    def __init__(self, max_batch, Hq, D, max_parts, device):
        self.max_parts = max_parts
        self.o = torch.empty((max_batch * Hq * max_parts * D,), dtype=torch.float32, device=device)
        self.m = torch.empty((max_batch * Hq * max_parts,), dtype=torch.float32, device=device)
        self.l = torch.empty((max_batch * Hq * max_parts,), dtype=torch.float32, device=device)
        # partition arrival counters of the in-launch combine (one per (sequence, kv head) <= Hq);
        # zero at rest: the last arriving workgroup resets its counter
        self.cnt = torch.zeros((max_batch * Hq,), dtype=torch.int32, device=device)


def paged_decode(q, k_cache, v_cache, block_tables, ctx_lens, part_size=512, workspace: DecodeWorkspace | None = None,
                 scale=None, out=None, order=None, warm=None):
    """q [B, Hq, D] (one new token per sequence) over the paged caches.  ``order`` (int32 [B], a
    permutation of the batch) is the order the (sequence, kv head) items are dispatched in: longest
    context first balances the two rounds of workgroups every CU runs at RAG batch sizes.  Any
    permutation is correct: the kernel bounds its partition walk by its own max over ctx_lens.

    ``warm`` = ``([(tensor, nbytes), ...up to 2], blocks)``: ``blocks`` workgroups appended to the
    launch read the first ``nbytes`` of each tensor into the Infinity Cache (the next projections'
    weights, while the latency-bound attention leaves the CUs idle); the output is unchanged."""
    B, Hq, D = q.shape
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if not q.is_cuda:
        return ref.paged_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale)
    _i32(ctx_lens)
    _i32(block_tables)
    expect_bf16_contig(q, k_cache, v_cache)
    Hkv, bs = k_cache.shape[1], k_cache.shape[2]
    expect(D in (64, 128), "decode head dim must be 64 or 128")
    expect(Hq % Hkv == 0 and Hq // Hkv <= 16, "GQA group must be <= 16")
    expect(part_size % 128 == 0, "part_size must be a multiple of 128")
    expect(block_tables.shape[0] >= B and ctx_lens.numel() >= B, "block table / ctx_lens rows < batch")
    max_parts = workspace.max_parts if workspace is not None else 1
    if workspace is None:
        # single partition covering the longest allowed context
        part_size = max(part_size, ((block_tables.shape[1] * bs + 127) // 128) * 128)
        ws_o = ws_m = ws_l = ws_c = None
    else:
        expect(workspace.o.numel() >= B * Hq * max_parts * D and workspace.cnt.numel() >= B * Hkv,
               "decode workspace too small")
        ws_o, ws_m, ws_l, ws_c = workspace.o, workspace.m, workspace.l, workspace.cnt
    out = torch.empty_like(q) if out is None else out
    if order is not None:
        _i32(order)
        expect(order.is_cuda and order.numel() >= B, "decode order must hold the batch")
    wargs = {}
    if warm is not None and warm[1] > 0:
        ranges, blocks = warm
        expect(1 <= len(ranges) <= 2 and 0 < blocks <= 1024, "warm: 1-2 ranges, 1-1024 workgroups")
        for i, (t, nb) in enumerate(ranges):
            expect(t.is_cuda and t.is_contiguous() and 0 < nb <= t.numel() * t.element_size() and nb % 16 == 0,
                   "warm range must be a 16-B multiple inside a contiguous device tensor")
            wargs[f"w{i}"], wargs[f"w{i}_bytes"] = ptr(t), int(nb)
        wargs["w_blocks"] = int(blocks)
    native().paged_decode_attention(ptr(q), ptr(k_cache), ptr(v_cache), ptr(block_tables), block_tables.shape[1], bs,
                                    ptr(ctx_lens), ptr(out), ptr(ws_o), ptr(ws_m), ptr(ws_l), ptr(ws_c), B, Hq, Hkv,
                                    D, int(part_size), int(max_parts), float(scale), stream(q), ptr(order), **wargs)
    return out


# ----------------------------------------------------------------------------------------------
# GEMM


GEMM256_MIN_M = 1024  # the phased 256x256 kernel from here on; the 128x128 kernel below


# gemm_mid from the first row: at M <= 191 the 128 x 128 kernel re-reads the weights per row tile
# and leaves most CUs idle -- Llama-3-8B qkv / o / gate_up / down at M = 129-187: 54 / 54 / 72 / 181
# us against 31 / 29 / 67 / 47 (profiles/small_prefill_r6.md; decode-sized prefill steps of the
# fragment-layout decoder stream instead, models/llama.py PREFILL_STREAM_MAX_M)
GEMM_MID_MIN_M = 1
GEMM_MID_FILL = 192  # gemm256 keeps a shape whose 256 x 256 tiles fill this many of the 256 CUs


def _g256_fill(M: int, N: int) -> tuple[int, float]:
    """(256 x 256 tiles, share of the last-wave-padded CU slots they fill) of gemm256 on 256 CUs."""
    tiles = -(-M // 256) * (N // 256)
    return tiles, tiles / (-(-tiles // 256) * 256)


def use_gemm_mid(M: int, N: int, K: int, lda: int) -> bool:
    """Mid-M shapes on fragment-layout weights go to the stream-K kernel (gemm_mid.hip) where the
    256 x 256 kernel would leave CUs idle: fewer than GEMM_MID_FILL tiles, or a last wave that
    leaves the chip under 70 % busy.  Measured (profiles/gemm_mid_r6.md): Llama-3-8B qkv / o / down
    at M = 384..2048 run 1.2-2.5x faster than the round-5 dispatch, gate_up at M = 640 / 768 (336
    tiles = 1.31 waves) 12 % faster than gemm256; gate_up at 384 / 512 / 1024 / 2048 and qkv at
    2048 stay on gemm256."""
    if M < GEMM_MID_MIN_M or N % 256 or not gemm_mid_ok(M, N, K, lda):
        return False
    tiles, fill = _g256_fill(M, N)
    return tiles < GEMM_MID_FILL or fill < 0.7


def use_gemm256(M: int, N: int, K: int, lda: int, ldb: int) -> bool:
    """Large-M shapes go to the phased 256x256 kernel (gemm256.hip), and so do shapes from M = 256 on
    whose 256 x 256 tiles fill >= GEMM_MID_FILL CUs (gate_up at M = 384-768: 84-161 us against
    105-184 on the 128 x 128 kernel, profiles/gemm_mid_r6.md)."""
    wide = M >= 256 and N % 256 == 0 and -(-M // 256) * (N // 256) >= GEMM_MID_FILL  # e.g. gate_up at M 256-1023
    return (M >= GEMM256_MIN_M or wide) and bool(native().gemm256_ok(M, N, K, lda, ldb))


def gemm_bt(A, B, bias=None, residual=None, epilogue=EPI_NONE, out_f32=False, row_group=None, q_group=None,
            allow=None, out=None, shuffled=False, n=None, b_group: int = 1):
    """C = A . B^T (+bias) (+act) (+residual) on MFMA; A [M, K], B [N, K] (K-contiguous rows).

    ``shuffled``: B is a ``shuffle_weights`` copy (the layout the decode GEMM streams, so a model
    keeps ONE copy of every projection) of ``B.shape[0]`` rows, of which the first ``n`` (default:
    all) are the matrix; ``b_group`` 8: a ``shuffle_weights(w, 8)`` copy."""
    expect(b_group == 1 or (shuffled and b_group == 8), "b_group: 1, or 8 with a shuffled copy")
    if shuffled:
        R = B.shape[0]
        N = R if n is None else int(n)
        expect(R % (16 * b_group) == 0 and B.shape[1] % 32 == 0 and B.is_contiguous() and R >= N,
               "shuffled B: contiguous [R, K] copy, R % (16 b_group) == 0, K % 32 == 0, R >= n")
        if not A.is_cuda:
            Bu = unshuffle_weights(B, b_group)[:N]
            return ref.gemm_bt(A, Bu, bias, residual, epilogue, out_f32, row_group, q_group, allow)
    if not A.is_cuda:
        return ref.gemm_bt(A, B, bias, residual, epilogue, out_f32, row_group, q_group, allow)
    expect(A.dtype == torch.bfloat16 and B.dtype == torch.bfloat16, "bf16 operands required")
    expect(A.stride(-1) == 1 and B.stride(-1) == 1, "operands must be K-contiguous")
    M, K = A.shape
    N = (B.shape[0] if n is None else int(n)) if shuffled else B.shape[0]
    expect(B.shape[1] == K, "inner dims mismatch")
    expect(K % 64 == 0 and N % 4 == 0, "gemm_bt needs K % 64 == 0 and N % 4 == 0")
    expect(A.stride(0) % 8 == 0 and B.stride(0) % 8 == 0, "row strides must be multiples of 8")
    if bias is not None:
        expect_bf16_contig(bias)
        expect(bias.numel() == N, "bias size mismatch")
    n_out = N // 2 if epilogue in (EPI_SWIGLU, EPI_SWIGLU8) else N
    if epilogue == EPI_SWIGLU:
        expect(N % 32 == 0 and not out_f32, "swiglu epilogue needs N % 32 == 0 and bf16 output")
    if epilogue == EPI_SWIGLU8:
        expect(N % 32 == 0 and not out_f32 and bias is None and residual is None,
               "swiglu8 epilogue needs N % 32 == 0, bf16 output, no bias / residual")
    if residual is not None:
        expect(residual.dtype == torch.bfloat16 and residual.stride(-1) == 1, "residual must be bf16 row-major")
        expect(tuple(residual.shape) == (M, n_out), "residual shape mismatch")
    allow_words = 0
    if allow is not None:
        expect(allow.dtype == torch.int32 and allow.is_contiguous() and allow.shape[0] == M, "allow mask shape")
        allow_words = allow.shape[1]
        expect(allow_words * 32 >= N, "allow mask too narrow")
    if row_group is not None:
        _i32(row_group)
        expect(row_group.numel() >= N, "row_group shorter than N")
    if q_group is not None:
        _i32(q_group)
        expect(q_group.numel() >= M, "q_group shorter than M")
    dtype = torch.float32 if out_f32 else torch.bfloat16
    if out is None:
        out = torch.empty((M, n_out), dtype=dtype, device=A.device)
    expect(out.dtype == dtype and out.stride(-1) == 1 and tuple(out.shape) == (M, n_out), "bad output buffer")
    plain = not out_f32 and row_group is None and q_group is None and allow is None
    if (plain and shuffled and N == B.shape[0] and bias is None and epilogue in (EPI_NONE, EPI_SWIGLU8)
            and use_gemm_mid(M, N, K, A.stride(0))):
        return gemm_mid(A, B, residual=residual, epilogue=epilogue, out=out, b_group=b_group)
    if (epilogue in (EPI_NONE, EPI_GELU, EPI_SWIGLU, EPI_SWIGLU8) and plain and (not shuffled or N == B.shape[0])
            and use_gemm256(M, N, K, A.stride(0), B.stride(0))):
        return _gemm256_into(A, B, out, bias, residual, epilogue, shuffled, b_group)
    native().gemm_bt(ptr(A), A.stride(0), ptr(B), B.stride(0), ptr(out), out.stride(0), ptr(bias), ptr(residual),
                     residual.stride(0) if residual is not None else 0, M, N, K, int(epilogue), int(out_f32),
                     ptr(row_group), ptr(q_group), ptr(allow), allow_words, stream(A),
                     B.shape[0] if shuffled else 0, int(b_group))
    return out


def _gemm256_into(A, B, out, bias, residual, epilogue, shuffled, b_group=1):
    M, K = A.shape
    native().gemm256(ptr(A), A.stride(0), ptr(B), B.stride(0), ptr(out), out.stride(0), ptr(bias), ptr(residual),
                     residual.stride(0) if residual is not None else 0, M, B.shape[0], K, int(epilogue), stream(A),
                     int(shuffled), int(b_group))
    return out


def gemm256(A, B, bias=None, residual=None, epilogue=EPI_NONE, shuffled=False, b_group: int = 1):
    """The phased 256x256 kernel directly, for any M (``gemm_bt`` takes it from M >= 1024):
    tests and benchmarks.  N % 256 == 0, K % 128 == 0."""
    M, K = A.shape
    N = B.shape[0]
    expect(A.is_cuda and A.dtype == torch.bfloat16 and B.dtype == torch.bfloat16, "bf16 CUDA operands required")
    expect(bool(native().gemm256_ok(M, N, K, A.stride(0), B.stride(0))), "gemm256: N % 256, K % 128, 16-B rows")
    expect(not shuffled or (B.is_contiguous() and B.shape[1] == K), "shuffled B must be a contiguous [N, K] copy")
    n_out = N // 2 if epilogue in (EPI_SWIGLU, EPI_SWIGLU8) else N
    out = torch.empty((M, n_out), dtype=torch.bfloat16, device=A.device)
    return _gemm256_into(A, B, out, bias, residual, epilogue, shuffled, b_group)


_MID_WS: dict = {}


def _mid_workspace(device: torch.device, s: int):
    """Partial-tile slabs + ready flags of ``gemm_mid``, one set per (device, stream): two streams
    running the kernel at once must not share them.  The flags are zero at rest (every launch leaves
    them zero)."""
    key = (device.index, s)
    ws = _MID_WS.get(key)
    if ws is None:
        nat = native()
        slabs = torch.empty((nat.gemm_mid_slab_bytes() // 4,), dtype=torch.float32, device=device)
        cnt = torch.zeros((1 << 16,), dtype=torch.int32, device=device)
        ws = _MID_WS[key] = (slabs, cnt)
    return ws


def gemm_mid_ok(M: int, N: int, K: int, lda: int) -> bool:
    """Shapes ``gemm_mid`` serves: N % 256, K % 64, ceil(M / 128) <= 32 (M <= 4096)."""
    return bool(native().gemm_mid_ok(M, N, K, lda)) and -(-M // 128) * (N // 256) <= (1 << 16)


def gemm_mid(A, B, residual=None, epilogue=EPI_NONE, out=None, variant: int = 0, b_group: int = 1):
    """C = A . B^T (+ residual) or SwiGLU over 8-row [gate | up] groups, B a ``shuffle_weights`` copy:
    the mid-M kernel (``gemm_mid.hip``: grouped stream-K, 128 x 256 tiles, in-launch owner combine) for
    M = 256..4096 (mixed serving steps, single prompts).  Bit-reproducible: the split-K partials are
    summed in a fixed order.  ``variant`` (A/B harness): 32 / 64 force the K-step; + 1000 leaves
    split tiles uncombined (timing only)."""
    M, K = A.shape
    N = B.shape[0]
    expect(A.is_cuda and A.dtype == torch.bfloat16 and B.dtype == torch.bfloat16, "bf16 CUDA operands required")
    expect(A.stride(-1) == 1 and B.is_contiguous() and B.shape[1] == K, "A K-contiguous, B a contiguous [N, K] copy")
    expect(epilogue in (EPI_NONE, EPI_SWIGLU8), "gemm_mid epilogues: none (+residual) or SwiGLU8")
    expect(gemm_mid_ok(M, N, K, A.stride(0)), "gemm_mid: N % 256, K % 64, M <= 4096, 16-B rows")
    expect(b_group in (1, 8), "gemm_mid: b_group 1 or 8")
    n_out = N // 2 if epilogue == EPI_SWIGLU8 else N
    if residual is not None:
        expect(epilogue == EPI_NONE and residual.dtype == torch.bfloat16 and residual.stride(-1) == 1
               and tuple(residual.shape) == (M, N), "residual must be bf16 [M, N]")
    if out is None:
        out = torch.empty((M, n_out), dtype=torch.bfloat16, device=A.device)
    expect(out.dtype == torch.bfloat16 and out.stride(-1) == 1 and tuple(out.shape) == (M, n_out), "bad output")
    s = stream(A)
    slabs, cnt = _mid_workspace(A.device, s)
    native().gemm_mid(ptr(A), A.stride(0), ptr(B), ptr(out), out.stride(0), ptr(residual),
                      residual.stride(0) if residual is not None else 0, M, N, K, int(epilogue), ptr(slabs),
                      slabs.numel() * 4, ptr(cnt), cnt.numel(), s, int(variant), int(b_group))
    return out


def score_candidates(A, B, thr, cap, row_group=None, q_group=None):
    """Filtered cosine scores of A [M, K] against B [N, K] that are >= thr[m], appended per query
    (no [M, N] score matrix).  -> (cand_val fp32 [M, cap] (-inf padded), cand_idx int32 [M, cap]
    (defined for the first count entries of a row only), count int32 [M]; count > cap means the
    list overflowed)."""
    expect(A.is_cuda and A.dtype == torch.bfloat16 and B.dtype == torch.bfloat16, "bf16 CUDA operands required")
    expect(A.stride(-1) == 1 and B.stride(-1) == 1 and A.stride(0) % 8 == 0 and B.stride(0) % 8 == 0,
           "operands must be K-contiguous with row strides % 8 == 0")
    M, K = A.shape
    N = B.shape[0]
    expect(B.shape[1] == K and K % 64 == 0 and N % 4 == 0, "score_candidates needs K % 64 == 0 and N % 4 == 0")
    expect(thr.dtype == torch.float32 and thr.is_contiguous() and thr.numel() >= M, "thr must be fp32 [M]")
    if row_group is not None:
        _i32(row_group)
        expect(row_group.numel() >= N, "row_group shorter than N")
    if q_group is not None:
        _i32(q_group)
        expect(q_group.numel() >= M, "q_group shorter than M")
    cand_val = torch.full((M, cap), float("-inf"), dtype=torch.float32, device=A.device)
    cand_idx = torch.empty((M, cap), dtype=torch.int32, device=A.device)
    cnt = torch.zeros(M, dtype=torch.int32, device=A.device)
    native().gemm_score_candidates(ptr(A), A.stride(0), ptr(B), B.stride(0), M, N, K, ptr(row_group), ptr(q_group),
                                   ptr(thr), ptr(cnt), ptr(cand_val), ptr(cand_idx), int(cap), stream(A))
    return cand_val, cand_idx, cnt


def score_candidates_shuffled(A, B_shuf, N, thr, cap, row_group=None, q_group=None):
    """``score_candidates`` over a copy of the rows in the ``shuffle_weights`` layout (``B_shuf``
    [R, K], R >= round_up(N, 128), R % 16 == 0): every 16-row x 32-k fragment is one coalesced 1 KB
    load (1..96 queries at K <= 768, 1..64 at K <= 1024: the persistent scan of index_scan.hip;
    more (K % 128 == 0): gemm256's candidate epilogue; the weight-streaming kernel's candidate
    epilogue otherwise)."""
    expect(A.is_cuda and A.dtype == torch.bfloat16 and B_shuf.dtype == torch.bfloat16, "bf16 CUDA operands required")
    M, K = A.shape
    expect(shuffled_scan_ok(M, K) and A.stride(-1) == 1 and A.stride(0) % 8 == 0, "queries need K % 128 == 0")
    expect(B_shuf.is_contiguous() and B_shuf.shape[1] == K, "shuffled copy [R, K]")
    expect(B_shuf.shape[0] % 16 == 0 and B_shuf.shape[0] >= -(-N // 128) * 128, "shuffled copy needs round_up(N, 128) rows")
    expect(thr.dtype == torch.float32 and thr.is_contiguous() and thr.numel() >= M, "thr must be fp32 [M]")
    if row_group is not None:
        _i32(row_group)
        expect(row_group.numel() >= N, "row_group shorter than N")
    if q_group is not None:
        _i32(q_group)
        expect(q_group.numel() >= M, "q_group shorter than M")
    cand_val = torch.full((M, cap), float("-inf"), dtype=torch.float32, device=A.device)
    cand_idx = torch.empty((M, cap), dtype=torch.int32, device=A.device)
    cnt = torch.zeros(M, dtype=torch.int32, device=A.device)
    native().score_candidates_shuf(ptr(A), A.stride(0), ptr(B_shuf), M, int(N), K, ptr(row_group), ptr(q_group),
                                   ptr(thr), ptr(cnt), ptr(cand_val), ptr(cand_idx), int(cap), stream(A),
                                   B_shuf.shape[0])
    return cand_val, cand_idx, cnt


def shuffled_scan_ok(M: int, K: int) -> bool:
    """Query counts / widths ``score_candidates_shuffled`` serves."""
    return M >= 1 and K % 128 == 0


def shuffle_rows_into(dst: torch.Tensor, rows: torch.Tensor, vals: torch.Tensor) -> None:
    """Writes ``vals`` [n, K] as rows ``rows`` of ``dst``, a [R, K] tensor in the ``shuffle_weights``
    layout (the incremental form of shuffle_weights, for copies that are updated in place)."""
    R, K = dst.shape
    v5 = dst.view(R // 16, K // 32, 4, 16, 8)
    rows = rows.to(dst.device, torch.long)
    v5[rows // 16, :, :, rows % 16, :] = vals.to(dst.dtype).reshape(-1, K // 32, 4, 8)


def _ref_stream_gemm(x, w, splits=1, epilogue=EPI_NONE, residual=None, norm_eps=0.0):
    """CPU semantics of ``stream_gemm`` (row-major ``w``): bf16 [M, N] / SwiGLU / fp32 slabs
    [S, M, N] whose sum is the product (slab 0 holds it, the others are zero).  ``norm_eps`` > 0:
    the product of the RMS-normalised rows of x (gains folded into w) before the epilogue."""
    if norm_eps > 0:
        xf = x.float()
        r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + norm_eps)
        y = xf @ w.float().t() * r
        if epilogue in (EPI_SWIGLU, EPI_SWIGLU8):
            grp = 16 if epilogue == EPI_SWIGLU else 8
            v = y.view(y.shape[0], -1, 2, grp)
            y = (torch.nn.functional.silu(v[:, :, 0]) * v[:, :, 1]).reshape(y.shape[0], -1)
        if splits > 1:
            return torch.cat([y[None], torch.zeros((splits - 1,) + tuple(y.shape))], 0)
        return y.to(torch.bfloat16)
    y = ref.gemm_bt(x, w, None, None, epilogue, out_f32=splits > 1)
    if splits > 1:
        return torch.cat([y[None], torch.zeros((splits - 1,) + tuple(y.shape), dtype=y.dtype)], 0)
    return y if residual is None else (y.float() + residual.float()).to(torch.bfloat16)


STREAM_KS = 128
STREAM_MAX_M = 256  # decode batches / prefill last-token LM heads up to this many rows stream the weights


def shuffle_weights(w: torch.Tensor, group: int = 1) -> torch.Tensor:
    """[N, K] row-major -> the same values in the fragment layout [N/16][K/32][64 lanes][8]: the
    16 x 32 tile an MFMA A fragment covers is 1 KB contiguous, in lane order (lane l = row l & 15,
    k 8 (l >> 4) .. + 8), so every weight load of the streaming kernel is one fully coalesced 1 KB
    read, and the prefill GEMMs' LDS-DMA copies whole blocks (gemm256 / gemm_bt ``shuffled``).
    ``group`` G > 1: the grouped form [N/(16G)][K/32][G][1 KB] -- the fragments of G consecutive
    16-row blocks adjacent for each 32-deep k chunk, so the decode GEMM's waves (one block each)
    stream neighbouring bytes (profiles/decode_stream_layout_r6.md); the kernels take it with
    ``w_group`` / ``b_group`` = G.  Returned with shape [N, K] (only the memory order changes)."""
    N, K = w.shape
    expect(N % (16 * group) == 0 and K % 32 == 0, "shuffle_weights needs N % (16 group) == 0 and K % 32 == 0")
    f = w.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4)
    if group > 1:
        f = f.reshape(N // (16 * group), group, K // 32, 512).permute(0, 2, 1, 3)
    return f.contiguous().view(N, K)


def unshuffle_weights(w: torch.Tensor, group: int = 1) -> torch.Tensor:
    """Inverse of ``shuffle_weights``."""
    N, K = w.shape
    if group > 1:
        w = w.reshape(N // (16 * group), K // 32, group, 512).permute(0, 2, 1, 3)
    return w.reshape(N // 16, K // 32, 4, 16, 8).permute(0, 3, 1, 2, 4).contiguous().view(N, K)


def stream_gemm(x, w, splits=1, epilogue=EPI_NONE, residual=None, out=None, nt=False, cfg=0, norm_eps: float = 0.0,
                slab_dtype=torch.float32, w_group: int = 1):
    """Decode GEMM y = x w^T on the warp-specialised streaming kernel (``stream_gemm.hip``): bf16
    [M, N] (optional residual add), SwiGLU [M, N/2] over 16- / 8-row interleaved [gate | up] rows, or
    fp32 K-slice slabs [S, M, N] (their sum is the product; consumers sum them in their prologue or
    ``slab_reduce`` does).  ``cfg`` picks the tile / ring configuration
    (``native().stream_gemm_bn(cfg)`` weight rows per workgroup); ``nt`` streams the weights with
    non-temporal loads.  ``norm_eps`` > 0: x is an un-normalised residual stream and w carries the
    RMSNorm gains in its columns; the kernel scales row m by rsqrt(mean(x[m]^2) + eps) (the
    consumer-side RMSNorm of small decode batches).  ``slab_dtype`` bf16: the split-K slabs are the
    partial sums rounded to bf16 (half the bytes for the producer and its consumer; the rounding the TP
    path's all-reduce input has).  On the CPU ``w`` is row-major."""
    if not x.is_cuda:
        y = _ref_stream_gemm(x, w, splits=splits, epilogue=epilogue, residual=residual, norm_eps=norm_eps)
        return y.to(slab_dtype) if splits > 1 else y
    expect(norm_eps <= 0 or residual is None, "the consumer RMSNorm takes no residual add")
    expect(x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16, "bf16 operands required")
    expect(x.stride(-1) == 1 and w.stride(-1) == 1, "operands must be K-contiguous")
    M, K = x.shape
    N = w.shape[0]
    bn = native().stream_gemm_bn(cfg)
    expect(bn > 0 and M <= native().stream_gemm_max_m(cfg), f"stream_gemm cfg {cfg}: bad config or M too large")
    expect(w.shape[1] == K and N % bn == 0 and K % (splits * STREAM_KS) == 0,
           f"stream_gemm needs N % {bn} == 0 and K % ({STREAM_KS}*splits) == 0")
    expect(x.stride(0) % 8 == 0 and w.stride(0) % 8 == 0, "row strides must be multiples of 8")
    if native().stream_gemm_shuffled(cfg):
        expect(w.is_contiguous(), "shuffled-layout configurations take a contiguous shuffle_weights() tensor")
    if splits > 1:
        expect(epilogue == EPI_NONE and residual is None, "split-K writes raw slabs")
        expect(slab_dtype in (torch.float32, torch.bfloat16), "slabs are fp32 or bf16")
        if out is None:
            out = torch.empty((splits, M, N), dtype=slab_dtype, device=x.device)
        expect(out.dtype == slab_dtype and out.is_contiguous() and tuple(out.shape) == (splits, M, N), "bad slabs")
        ldo = N
    else:
        n_out = N // 2 if epilogue in (EPI_SWIGLU, EPI_SWIGLU8) else N
        if residual is not None:
            expect(epilogue == EPI_NONE and residual.dtype == torch.bfloat16 and residual.stride(-1) == 1
                   and tuple(residual.shape) == (M, N), "residual must be bf16 [M, N]")
        if epilogue == EPI_SWIGLU:
            expect(bn % 32 == 0, f"stream_gemm cfg {cfg}: EPI_SWIGLU needs 32-row tiles (use EPI_SWIGLU8)")
        if out is None:
            out = torch.empty((M, n_out), dtype=torch.bfloat16, device=x.device)
        expect(out.dtype == torch.bfloat16 and out.stride(-1) == 1 and tuple(out.shape) == (M, n_out), "bad output")
        ldo = out.stride(0)
    native().stream_gemm(ptr(x), x.stride(0), ptr(w), w.stride(0), ptr(out), ldo, ptr(residual),
                         residual.stride(0) if residual is not None else 0, M, N, K, splits, int(epilogue), stream(x),
                         int(bool(nt)), int(cfg), float(norm_eps), int(splits > 1 and out.dtype == torch.bfloat16),
                         int(w_group))
    return out


def slab_reduce(slabs, residual=None, out=None):
    """fp32 / bf16 slabs [S, M, N] -> bf16 [M, N] (fp32 sum rounded to bf16, then + residual)."""
    if not slabs.is_cuda:
        y = slabs.float().sum(0).to(torch.bfloat16)
        return y if residual is None else (y.float() + residual.float()).to(torch.bfloat16)
    S, M, N = slabs.shape
    expect(slabs.dtype in (torch.float32, torch.bfloat16) and slabs.is_contiguous() and N % 8 == 0, "bad slabs")
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=slabs.device)
    if residual is not None:
        expect(residual.dtype == torch.bfloat16 and tuple(residual.shape) == (M, N) and residual.stride(-1) == 1,
               "residual must be bf16 [M, N]")
    native().slab_reduce(ptr(out), out.stride(0), ptr(slabs), S, M, N, ptr(residual),
                         residual.stride(0) if residual is not None else 0, stream(slabs),
                         int(slabs.dtype == torch.bfloat16))
    return out


def interleave_gate_up(w_gate: torch.Tensor, w_up: torch.Tensor, group: int = 16) -> torch.Tensor:
    """[F, H] gate and up weights -> [2F, H] interleaved in ``group``-row groups [g | u | g | u ...]
    (16: the layout the SWIGLU epilogue of gemm_bt / gemm256 consumes; 8: EPI_SWIGLU8)."""
    Fd, H = w_gate.shape
    assert Fd % group == 0
    g = w_gate.reshape(Fd // group, group, H)
    u = w_up.reshape(Fd // group, group, H)
    return torch.stack([g, u], dim=1).reshape(2 * Fd, H).contiguous()


def regroup_gate_up(w: torch.Tensor, src: int = 16, dst: int = 8) -> torch.Tensor:
    """Re-interleave [2F, H] gate|up weights from ``src``-row to ``dst``-row groups."""
    n2, H = w.shape
    v = w.reshape(n2 // (2 * src), 2, src, H)
    gate, up = v[:, 0].reshape(n2 // 2, H), v[:, 1].reshape(n2 // 2, H)
    return interleave_gate_up(gate, up, dst)


# ----------------------------------------------------------------------------------------------
# selection


SAMPLE_FAST_MAX_K = 64
_CHUNK = 256 * 32


def sample_workspace(rows: int, vocab: int, device) -> torch.Tensor:
    ncand = -(-vocab // _CHUNK) * SAMPLE_FAST_MAX_K
    return torch.empty((rows * ncand * 8,), dtype=torch.uint8, device=device)


def sample_tokens(logits, temperature, top_k, top_p, seed: int, counters, generator=None, out=None,
                  fast: bool | None = None, workspace: torch.Tensor | None = None):
    """temperature / top_k (int32) / top_p per row; counters int64 per row (advanced in-kernel).

    ``fast`` (every row has 0 < top_k <= 64, the reference's 50 included) selects the two-stage kernel:
    per-chunk register-resident top-64 over many workgroups, then a per-row merge + top-p + sample."""
    if not logits.is_cuda:
        return ref.sample_hf(logits, temperature, top_k, top_p, generator)
    rows, vocab = logits.shape
    expect(logits.stride(-1) == 1, "logits rows must be contiguous")
    expect(logits.dtype in (torch.float32, torch.bfloat16), "logits must be fp32 or bf16")
    expect(temperature.dtype == torch.float32 and temperature.numel() >= rows, "temperature")
    expect(top_p.dtype == torch.float32 and top_p.numel() >= rows, "top_p")
    _i32(top_k)
    expect(counters.dtype == torch.int64 and counters.numel() >= rows, "counters")
    out = torch.empty((rows,), dtype=torch.int32, device=logits.device) if out is None else out
    if fast is None:
        fast = False
    ncand = -(-vocab // _CHUNK) * SAMPLE_FAST_MAX_K
    if fast and ncand <= 1024:
        ws = workspace if workspace is not None else sample_workspace(rows, vocab, logits.device)
        expect(ws.numel() >= rows * ncand * 8, "sampling workspace too small")
        native().sample_tokens_2stage(ptr(logits), int(logits.dtype == torch.float32), logits.stride(0), rows, vocab,
                                      ptr(temperature), ptr(top_k), ptr(top_p), int(seed) & ((1 << 64) - 1),
                                      ptr(counters), ptr(out), ptr(ws), ws.numel(), stream(logits))
    else:
        native().sample_tokens(ptr(logits), int(logits.dtype == torch.float32), logits.stride(0), rows, vocab,
                               ptr(temperature), ptr(top_k), ptr(top_p), int(seed) & ((1 << 64) - 1), ptr(counters),
                               ptr(out), 0, stream(logits))
    return out


def mask_logits(logits, mask, row_flags, vocab: int | None = None, word_offset: int = 0):
    """In place: logits[r, t] = -inf where bit t of ``mask[r]`` (int32 words, bit t % 32 of word
    t // 32) is clear, for the rows whose ``row_flags[r]`` (int32) is non-zero (JSON-constrained
    decoding).  Vocab-parallel slices: the first ``vocab`` columns of ``logits`` are tokens
    32 * ``word_offset`` ... (mask words ``word_offset`` ...).  Returns ``logits``."""
    rows = logits.shape[0]
    vocab = logits.shape[1] if vocab is None else int(vocab)
    words = -(-vocab // 32)
    expect(mask.dtype == torch.int32 and mask.is_contiguous() and mask.shape[0] >= rows
           and mask.shape[1] >= word_offset + words, "mask: int32 [rows, >= ceil(vocab / 32) words past the offset]")
    if not logits.is_cuda:
        m = mask[:rows, word_offset:word_offset + words]
        bits = (m.view(torch.int32).unsqueeze(-1) >> torch.arange(32, dtype=torch.int32)) & 1
        allow = bits.reshape(rows, -1)[:, :vocab].bool() | (row_flags[:rows] == 0).unsqueeze(1)
        logits[:, :vocab].masked_fill_(~allow, float("-inf"))
        return logits
    expect(logits.stride(-1) == 1 and logits.dtype in (torch.float32, torch.bfloat16), "logits: fp32/bf16 rows")
    _i32(row_flags)
    native().mask_logits(ptr(logits), int(logits.dtype == torch.float32), logits.stride(0), rows, vocab,
                         ptr(mask) + 4 * int(word_offset), words, ptr(row_flags), stream(logits), mask.stride(0))
    return logits


def sample_candidates(logits, vocab: int, index_base: int = 0, out=None):
    """Stage 1 of vocab-parallel sampling: each 8192-token chunk's top-64 of the first ``vocab``
    columns of ``logits`` as (order-preserving uint32 key, token id + ``index_base``) -> int32
    [2, rows, ncand] (keys, then ids).  The TP ranks all-gather these and ``sample_merge`` draws
    from the union (GPU only)."""
    expect(logits.is_cuda and logits.stride(-1) == 1 and logits.dtype in (torch.float32, torch.bfloat16),
           "logits: CUDA fp32/bf16 rows")
    rows = logits.shape[0]
    ncand = sample_candidates_per_row(vocab)
    if out is None:
        out = torch.empty((2, rows, ncand), dtype=torch.int32, device=logits.device)
    # (a row slice of a larger [2, R, ncand] buffer is fine: each half is rows x ncand contiguous)
    expect(out.dtype == torch.int32 and tuple(out.shape) == (2, rows, ncand) and out.stride(2) == 1
           and out.stride(1) == ncand, "candidates: int32 [2, rows, ncand] with contiguous halves")
    native().sample_candidates(ptr(logits), int(logits.dtype == torch.float32), logits.stride(0), rows, int(vocab),
                               int(index_base), ptr(out[0]), ptr(out[1]), ncand, stream(logits))
    return out


def sample_candidates_per_row(vocab: int) -> int:
    return -(-int(vocab) // _CHUNK) * SAMPLE_FAST_MAX_K


def sample_merge(cands, temperature, top_k, top_p, seed: int, counters, vocab: int, out=None):
    """Stage 2 of vocab-parallel sampling: ``cands`` int32 [2, rows, n] (every rank's
    ``sample_candidates`` side by side along n, n <= 1024) -> sorted top-k -> HF top-p ->
    multinomial with the per-row counter RNG (advanced in-kernel): the replicated head's draw."""
    two, rows, n = cands.shape
    expect(two == 2 and n <= 1024 and cands.dtype == torch.int32 and cands.is_contiguous(),
           "candidates: contiguous int32 [2, rows, <= 1024]")
    out = torch.empty((rows,), dtype=torch.int32, device=cands.device) if out is None else out
    _i32(top_k)
    native().sample_merge(ptr(cands[0]), ptr(cands[1]), n, rows, int(vocab), ptr(temperature), ptr(top_k), ptr(top_p),
                          int(seed) & ((1 << 64) - 1), ptr(counters), ptr(out), stream(cands))
    return out


def topk_rows(scores, k, index_base=0, want_global=False):
    """Exact per-row top-k of fp32 scores, sorted descending.  Returns (values, idx int32) or, with
    ``want_global``, (values, idx + index_base as int64).  Long rows use the two-stage kernel."""
    rows, n = scores.shape
    expect(1 <= k <= min(n, 1024), "1 <= k <= min(n, 1024)")
    if rows == 0:  # e.g. a rank with no queries in a sharded search (an empty view's strides are arbitrary)
        return (torch.empty((0, k), dtype=torch.float32, device=scores.device),
                torch.empty((0, k), dtype=torch.int64 if want_global else torch.int32, device=scores.device))
    if not scores.is_cuda:
        v, i = ref.topk_rows(scores, k)
        return (v, i.long() + index_base) if want_global else (v, i)
    expect(scores.dtype == torch.float32 and scores.stride(-1) == 1, "scores must be fp32 with contiguous rows")
    vals = torch.empty((rows, k), dtype=torch.float32, device=scores.device)
    if want_global:
        idx = torch.empty((rows, k), dtype=torch.int64, device=scores.device)
        i32, i64 = 0, ptr(idx)
    else:
        idx = torch.empty((rows, k), dtype=torch.int32, device=scores.device)
        i32, i64 = ptr(idx), 0
    if n >= 4 * _CHUNK:
        kc = -(-k // 64) * 64
        ncand = -(-n // _CHUNK) * kc
        ws = torch.empty((rows * ncand * 8,), dtype=torch.uint8, device=scores.device)
        native().topk_rows_2stage(ptr(scores), scores.stride(0), rows, n, k, ptr(vals), i32, int(index_base), i64,
                                  ptr(ws), ws.numel(), stream(scores))
    else:
        native().topk_rows(ptr(scores), scores.stride(0), rows, n, k, ptr(vals), i32, int(index_base), i64,
                           stream(scores))
    return vals, idx


def linear(x, w, b=None, residual=None, act=None):
    """y = x W^T (+b) (+act) (+residual) on the native MFMA GEMMs (``gemm_bt``: the phased 256x256
    kernel for large token counts, the 128x128 kernel otherwise), epilogues fused.

    Widths the kernels do not tile (K % 64, N % 4) are zero-padded to the next native shape (zero
    k-columns add nothing to a dot product; padded output columns are sliced off), so every GPU
    call runs the native kernel -- there is no torch fallback (``ops/_lib.py`` dispatch rule)."""
    epi = {None: EPI_NONE, "gelu": EPI_GELU, "swiglu": EPI_SWIGLU}[act]
    if not x.is_cuda:
        return ref.gemm_bt(x, w, b, residual, epi)
    K, N = x.shape[-1], w.shape[0]
    expect(epi != EPI_SWIGLU or N % 32 == 0, "swiglu linear needs 16-row [gate | up] groups (N % 32 == 0)")
    x2 = x.reshape(-1, K)
    r2 = residual.reshape(x2.shape[0], -1) if residual is not None else None
    pk, pn = (-K) % 64, (-N) % 4
    if pk or pn:
        x2 = F.pad(x2, (0, pk)) if pk else x2
        w = F.pad(w, (0, pk, 0, pn))
        b = F.pad(b, (0, pn)) if (b is not None and pn) else b
        r2 = F.pad(r2, (0, pn)) if (r2 is not None and pn) else r2
    y = gemm_bt(x2, w, b, r2, epi)
    if pn:
        y = y[:, :N].contiguous()
    return y.view(*x.shape[:-1], y.shape[-1])
