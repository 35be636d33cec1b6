"""Llama-3 family decoder on the native kernels with a paged KV cache and tensor parallelism.

Replaces HF ``AutoModelForCausalLM.generate`` of the reference (ai/providers/transformers.py:35-94).
One forward serves both phases:

  * prefill (packed variable-length prompt chunks; flash attention reads K/V from the paged cache,
    so chunked prefill and cached shared prefixes need no special path);
  * decode (one token per running sequence; split-K paged decode attention), capturable in a HIP
    graph because every op enqueues on the current stream with fixed shapes.

Per layer:  RMSNorm(+residual) -> QKV GEMM -> RoPE + KV-cache write -> attention -> O GEMM
[-> TP all-reduce] -> RMSNorm(+residual) -> gate|up GEMM (+fused SwiGLU) -> down GEMM
[-> TP all-reduce].  Under TP each rank owns Hq/tp query heads, Hkv/tp KV heads and F/tp MLP
columns (Megatron split); the two all-reduces per layer run on the RCCL process group.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .. import ops
from ..ops import reference as ref
from .configs import DecoderConfig


@dataclass
class DecoderLayer:
    """One layer's tensors.  On the GPU the four projections are held ONCE, in the
    ``ops.shuffle_weights`` fragment layout, which the decode GEMM (stream_gemm) streams and the
    prefill GEMMs (gemm256 / gemm_bt ``shuffled``) stage by LDS-DMA; on the CPU they are row-major."""

    attn_norm: torch.Tensor
    qkv_w: torch.Tensor
    o_w: torch.Tensor
    mlp_norm: torch.Tensor
    gate_up_w: torch.Tensor  # [gate 8 | up 8] row groups (interleaved) or [gate; up] (stacked)
    down_w: torch.Tensor


@dataclass
class AttnMeta:
    """Per-forward batch description (device tensors, fixed shapes in decode graphs)."""

    decode: bool
    positions: torch.Tensor  # int32 [T]
    slots: torch.Tensor  # int64 [T] cache slot of each token (<0 = padding)
    block_tables: torch.Tensor  # int32 [B, max_blocks]
    ctx_lens: torch.Tensor  # int32 [B] total tokens in cache after this step
    cu_q: torch.Tensor | None = None  # int32 [B+1] (prefill)
    max_q: int = 1
    workspace: ops.DecodeWorkspace | None = None
    part_size: int = 512
    # mixed step: the LAST n_decode tokens are single-token decode rows (one per sequence) with their
    # own block tables / context lengths; the tokens before them are prefill chunks described above
    n_decode: int = 0
    dec_block_tables: torch.Tensor | None = None
    dec_ctx_lens: torch.Tensor | None = None
    order: torch.Tensor | None = None  # int32 [B] decode attention dispatch order (longest context first;
    # of the decode rows in a mixed step)


class _Partial:
    """This rank's un-reduced TP partial sum of a row-parallel projection (fp32 split-K slabs or
    bf16): the all-reduce is still due and runs fused into the RMSNorm that consumes it
    (``LlamaModel._norm``: one launch instead of slab_reduce + all-reduce + rmsnorm)."""

    __slots__ = ("t",)

    def __init__(self, t: torch.Tensor):
        self.t = t


class KVCache:
    """Paged KV cache: per layer [num_blocks, Hkv_local, block_size, D] for K and for V."""

    def __init__(self, layers, num_blocks, kv_heads, block_size, head_dim, device, dtype=torch.bfloat16):
        self.num_blocks, self.block_size = num_blocks, block_size
        self.k = torch.zeros((layers, num_blocks, kv_heads, block_size, head_dim), device=device, dtype=dtype)
        self.v = torch.zeros_like(self.k)

    @staticmethod
    def bytes_per_block(layers, kv_heads, block_size, head_dim, dtype=torch.bfloat16):
        return 2 * layers * kv_heads * block_size * head_dim * torch.finfo(dtype).bits // 8


class LlamaModel:
    # rows of a vocab-parallel LM head shard are padded to a multiple of this (every stream_gemm
    # tile height and the fragment layout divide it); the pad rows are zero and never sampled
    VOCAB_PAD = 384

    def __init__(self, cfg: DecoderConfig, weights: dict, device, tp_group=None, tp_size: int = 1,
                 interleaved_mlp: bool = False, fragment_layout: bool = True, consume: bool = False,
                 tp_rank: int | None = None, vocab_parallel: bool = True, small_norm_fused: bool | None = None):
        """``consume``: the entries of ``weights`` are popped as the model takes them over, so each
        original is freed as soon as its fragment-layout copy exists (peak HBM = model + one
        tensor: 70B at TP 1 needs it, 2 x 140 GB would not fit in 288 GB).

        ``vocab_parallel`` (TP > 1): the LM head is split by vocabulary rows, rank r keeping tokens
        [r V/tp, (r+1) V/tp) (a replicated head streamed the whole 2.1 GB 70B head
        on every rank every step).  Each rank then produces the logits of its slice only; the engine
        samples from the all-gathered per-slice candidates (``ops.sample_candidates`` /
        ``sample_merge``).  Needs V % (32 tp) == 0 (whole JSON-mask words per slice); otherwise the
        head stays replicated."""
        self.cfg = cfg
        self.device = torch.device(device)
        if tp_rank is None:
            tp_rank = 0
            if tp_size > 1:
                import torch.distributed as dist

                tp_rank = dist.get_rank(tp_group) if dist.is_initialized() else 0
        self.tp_group, self.tp_size, self.tp_rank = tp_group, tp_size, tp_rank
        V = cfg.vocab_size
        # (the merged candidate set, tp x 64 per 8192-token chunk of a slice, must fit the merge
        # kernel's 1024 entries: true for Llama-3's 128256 tokens at tp 2 / 4 / 8)
        self.vocab_parallel = (bool(vocab_parallel) and tp_size > 1 and V % (32 * tp_size) == 0
                               and tp_size * -(-(V // tp_size) // 8192) * 64 <= 1024)
        self.vocab_local = V // tp_size if self.vocab_parallel else V
        self.vocab_start = tp_rank * self.vocab_local if self.vocab_parallel else 0
        self.hq = cfg.heads // tp_size
        self.hkv = cfg.kv_heads // tp_size
        self.interleaved_mlp = interleaved_mlp  # gate_up rows in 8-row [gate | up] groups (EPI_SWIGLU8)
        # One copy of every projection, in the fragment layout both GEMM families read (VERDICT r2
        # "stop paying HBM twice": the decode-only shuffled copies were +15 GB for Llama-3-8B and
        # disabled the streaming decode for 70B at TP 1).  The LM head too; a tied embedding table
        # keeps its row-major copy for the gather.
        # (``fragment_layout=False``: row-major weights on the GPU too, every projection on the
        # 128x128 / phased 256x256 GEMMs -- the comparison path of tests/test_models_gpu.py)
        self.frag = fragment_layout and self.device.type == "cuda" and self._fragment_ok(weights)
        take = weights.pop if consume else weights.__getitem__

        self.proj_group = {}

        def fmt(name, t):
            """The decoder's one copy of projection ``name``: the fragment layout, grouped per
            ``PROJ_GROUPS`` where the shape allows (layer 0 decides for every layer)."""
            if not self.frag:
                return t
            if name not in self.proj_group:
                g = self.PROJ_GROUPS.get(name, 1)
                self.proj_group[name] = g if (t.shape[0] % (16 * g) == 0 and t.numel() * 2 < (1 << 31)) else 1
            return ops.shuffle_weights(t, self.proj_group[name])

        self.embed = take("embed").to(self.device)
        self.final_norm = take("final_norm").to(self.device)
        head = take("lm_head").to(self.device) if "lm_head" in weights else self.embed
        if self.vocab_parallel:
            head = head[self.vocab_start:self.vocab_start + self.vocab_local]
            pad = (-self.vocab_local) % self.VOCAB_PAD if self.frag else 0
            if pad:
                head = torch.cat([head, head.new_zeros((pad, head.shape[1]))])
            head = head.contiguous()
        self.lm_head = ops.shuffle_weights(head) if self.frag else head
        del head
        # ``small_norm_fused`` (opt-in, measured slower: profiles/decode_small_r5.md): the attention /
        # MLP RMSNorm gains move into the columns of the projection each norm feeds
        # (rmsnorm(x) g W^T = rmsnorm(x) (W diag g)^T) and the norms run with unit gains, so small
        # decode batches can normalise inside the consumer GEMM (``_layer_small``).  The fold is one
        # more bf16 rounding of W diag(g), so the default model keeps the reference norm -> GEMM
        # order and does not fold.
        if small_norm_fused is not None:
            self.small_norm_fused = bool(small_norm_fused)
        self.fold_norms = self.frag and self.small_norm_fused
        self.layers = []
        for i in range(cfg.layers):
            an = take(f"l{i}.attn_norm").to(self.device)
            mn = take(f"l{i}.mlp_norm").to(self.device)
            qkv_w, gu_w = take(f"l{i}.qkv_w").to(self.device), take(f"l{i}.gate_up_w").to(self.device)
            if self.fold_norms:
                qkv_w, an = self._fold(qkv_w, an), torch.ones_like(an)
                gu_w, mn = self._fold(gu_w, mn), torch.ones_like(mn)
            o_w, down_w = take(f"l{i}.o_w").to(self.device), take(f"l{i}.down_w").to(self.device)
            self.layers.append(DecoderLayer(an, fmt("qkv", qkv_w), fmt("o", o_w), mn, fmt("gate_up", gu_w),
                                            fmt("down", down_w)))
            del o_w, down_w
            del qkv_w, gu_w
        if self.frag and consume:
            torch.cuda.empty_cache()

        self.custom_ar = None  # parallel.custom_allreduce.CustomAllReduce (set by the engine)
        # TP all-reduces issued from Python: one-shot IPC vs the process group (RCCL / gloo); a call
        # captured into a decode graph counts once, at capture, not per replay
        self.ar_counts = {"ipc": 0, "ipc_fused_norm": 0, "group": 0}
        inv = ref.llama3_inv_freq(cfg.head_dim, cfg.rope_theta, cfg.rope_scaling)
        self.cos_sin = ref.rope_cos_sin(inv, cfg.max_position).to(self.device)

    @staticmethod
    def _fold(w: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
        """W diag(g) (unit gains, e.g. random init: W itself)."""
        if bool(torch.all(g == 1)):
            return w
        return (w.float() * g.float()[None, :]).to(w.dtype)

    def full_logits(self, local: torch.Tensor) -> torch.Tensor:
        """All-gather the vocab-parallel slices of every TP rank -> [n, V] (the CPU sampling path
        and tests; the GPU path gathers candidates instead)."""
        if not self.vocab_parallel:
            return local
        import torch.distributed as dist

        src = local[:, :self.vocab_local].contiguous()
        staged = src.is_cuda and dist.get_backend(self.tp_group) != "nccl"  # gloo rehearsals on one GPU
        if staged:
            src = src.cpu()
        parts = [torch.empty_like(src) for _ in range(self.tp_size)]
        dist.all_gather(parts, src, group=self.tp_group)
        return torch.cat(parts, 1).to(local.device)

    def set_proj_group(self, name: str, group: int) -> None:
        """Re-lay every layer's copy of projection ``name`` (qkv / o / gate_up / down) as
        ``shuffle_weights(w, group)``, in place (captured graphs keep their pointers but bake the group
        in: re-capture after a change).  A/B harness."""
        old = self.proj_group.get(name, 1)
        if not self.frag or group == old:
            return
        for L in self.layers:
            w = getattr(L, name + "_w")
            if w.shape[0] % (16 * group):
                raise ValueError(f"{name}: {w.shape[0]} rows are not whole groups of {group}")
            w.copy_(ops.shuffle_weights(ops.unshuffle_weights(w, old), group))
        self.proj_group[name] = group

    def _fragment_ok(self, weights: dict) -> bool:
        keys = ["lm_head" if "lm_head" in weights else "embed"] + [
            f"l{i}.{n}" for i in range(self.cfg.layers) for n in ("qkv_w", "o_w", "gate_up_w", "down_w")]
        return self.interleaved_mlp and all(weights[k].shape[0] % 16 == 0 and weights[k].shape[1] % 64 == 0
                                            for k in keys)

    @property
    def dtype(self):
        return self.embed.dtype

    def _all_reduce(self, x):
        """TP partial sums: the one-shot IPC all-reduce for decode-sized messages when the engine
        attached one (``custom_ar``), RCCL otherwise (prefill, CPU/gloo)."""
        if self.tp_size > 1:
            ar = self.custom_ar
            if ar is not None and ar.eligible(x):
                self.ar_counts["ipc"] += 1
                return ar.all_reduce(x)
            import torch.distributed as dist

            self.ar_counts["group"] += 1
            dist.all_reduce(x, group=self.tp_group)
        return x

    # stream_gemm.hip configurations (shuffled weights): BN 128 rows per workgroup at M <= 64 (13)
    # and M <= 128 (10).  Whole-chip tilings at M 65..128: gate_up's 28672 rows / 112 make exactly
    # 256 workgroups where BN 128 left 32 of the 256 CUs idle (cfg 20: 54.9 -> 51.5 us cold); the LM
    # head uses 192-row tiles (cfg 28: 2/3 of the X staging per weight byte, 228.7 -> 221.3 us).
    # qkv at 96 rows x 4 K-slices (cfg 21) measured slower than BN 128 x 4 (17.1 vs 15.8 us).
    # Decode batches of 129..256 rows: 64-row tiles, 2 k-groups x 4 row groups (cfg 27; M = 256:
    # qkv 27.4 / o 18.6 / gate_up 98.7 / down 49.2 us against 32.4 / 25.8 / 104 / 55 for two
    # M = 128 passes, profiles/decode_round2.md).
    STREAM_CFG_M16, STREAM_CFG_M32, STREAM_CFG_M64, STREAM_CFG_M128, STREAM_CFG_M256 = 30, 31, 13, 10, 27
    STREAM_WIDE = {"gate_up": 20, "lm_head": 28}
    STREAM_MAX_M = ops.STREAM_MAX_M
    PREFILL_STREAM_MAX_M = 128  # prefill steps of at most this many tokens stream too (0: off)

    def _stream_cfg(self, name: str, M: int, N: int) -> int:
        nat = ops.native()
        if M > 128 and name == "gate_up":
            # decode batches of 129..256: gate_up (+SwiGLU8) on the mid-M GEMM, 67-72 us against 90-96
            # on the M <= 256 streaming tiles (profiles/small_prefill_r6.md); qkv / o / down stream
            return -1
        if M > 128:
            cfg = self.STREAM_CFG_M256
        elif M <= 16 and N % nat.stream_gemm_bn(self.STREAM_CFG_M16) == 0:
            cfg = self.STREAM_CFG_M16
        elif M <= 32 and N % nat.stream_gemm_bn(self.STREAM_CFG_M32) == 0:
            cfg = self.STREAM_CFG_M32
        elif M <= 64:
            cfg = self.STREAM_CFG_M64
        else:
            cfg = self.STREAM_WIDE.get(name)
            if cfg is None or N % nat.stream_gemm_bn(cfg):
                cfg = self.STREAM_CFG_M128
        return cfg if N % nat.stream_gemm_bn(cfg) == 0 else -1

    @staticmethod
    def _stream_splits(N: int, K: int, bn: int = 128) -> int:
        """K-slices for stream_gemm: the fewest that give >= 192 workgroups of ``bn`` weight rows."""
        tiles, best = N // bn, 1
        for s in (1, 2, 4, 8, 16):
            if K % (128 * s):
                break
            best = s
            if tiles * s >= 192:
                break
        return best

    def _stream_choice(self, name: str, M: int, N: int, K: int) -> tuple[int, int]:
        """(stream_gemm cfg, K-slices) of a decode projection; cfg -1 = not streamable.  (The tuning
        harness benchmarks/decode_ab.py overrides this in a subclass.)"""
        cfg = self._stream_cfg(name, M, N)
        if cfg < 0 or K % 128:
            return -1, 1
        return cfg, self._stream_splits(N, K, ops.native().stream_gemm_bn(cfg))

    # Projections held in the grouped fragment layout (shuffle_weights(w, G): the G row blocks of
    # each 16 G-row group adjacent per 32-deep k chunk), so the decode GEMM's waves (one block each)
    # stream neighbouring bytes; every GEMM reading a copy takes its group (``proj_group``).  gate_up
    # at 8: batch-128 decode step 7.31 -> 7.23 ms (profiles/decode_stream_layout_r6.md)
    PROJ_GROUPS = {"gate_up": 8}

    # Split-K slabs of the decode projections as bf16 (the partial sums rounded once, as the TP path
    # hands them to its all-reduce) instead of fp32: half the bytes the producer writes and the
    # RMSNorm / RoPE consumers read; batch-128 decode step 7.503 -> 7.351 ms (benchmarks/decode_ab.py
    # slab32,slab16; profiles/decode_slab_r6.md).  TP keeps fp32: its fused all-reduce + norm sums
    # fp32 slabs.
    slab_bf16 = True

    def _proj(self, x, w, dec: bool, allow_slabs: bool = True, name: str = "", epilogue=ops.EPI_NONE):
        """One projection.  Decode-sized batches (``dec``) stream the fragment-layout weights
        through stream_gemm, as fp32 split-K slabs when a consumer sums them (RMSNorm, the decode
        attention's RoPE prologue) and ``allow_slabs``; everything else runs the MFMA GEMM on the
        same copy (gemm256 for large token counts, the 128x128 kernel below that)."""
        if not x.is_cuda:
            if epilogue == ops.EPI_SWIGLU8 or (epilogue == ops.EPI_NONE and name == "gate_up"):
                y = ops.linear(x, w)
                return ops.silu_mul(y, group=8 if self.interleaved_mlp else 0)
            return ops.linear(x, w)
        grp = self.proj_group.get(name, 1)
        if dec and self.frag:
            cfg, s = self._stream_choice(name, x.shape[0], w.shape[0], w.shape[1])
            if cfg >= 0:
                if epilogue != ops.EPI_NONE:
                    return ops.stream_gemm(x, w, epilogue=epilogue, nt=True, cfg=cfg, w_group=grp)
                sd = torch.bfloat16 if (self.slab_bf16 and self.tp_size == 1) else torch.float32
                out = ops.stream_gemm(x, w, splits=s, cfg=cfg, nt=True, slab_dtype=sd, w_group=grp)
                return ops.slab_reduce(out) if (s > 1 and not allow_slabs) else out
        return ops.gemm_bt(x, w, epilogue=epilogue, shuffled=self.frag, b_group=grp)

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: KVCache) -> torch.Tensor:
        """ids int32 [T] -> final hidden states [T, H] (after the last RMSNorm)."""
        cfg = self.cfg
        D = cfg.head_dim
        T = ids.numel()
        x = ops.embed_gather(ids, self.embed)
        # decode-sized batches stream the weights through the split-K MFMA kernel; its fp32 slabs
        # are summed by the consumers (RoPE/KV write, RMSNorm) instead of a separate reduction.  So
        # do short prefill steps (an interactive prompt, the tail of a batch): at T <= 128 the MFMA
        # tiles read every weight for a handful of rows (qkv / o / gate_up / down 54 / 54 / 65 /
        # 183 us against 16-21 / 15-19 / 42-49 / 27-32 streamed, profiles/small_prefill_r6.md)
        small_pf = (not meta.decode and not meta.n_decode and T <= self.PREFILL_STREAM_MAX_M and self.frag
                    and self.tp_size == 1)
        sk = (meta.decode and T <= self.STREAM_MAX_M or small_pf) and x.is_cuda
        if sk and meta.decode and T <= self.SMALL_FUSED_MAX_M and self.small_norm_fused and self.fold_norms and self.tp_size == 1:
            h = x  # the residual stream itself: no RMSNorm launches (``_layer_small``)
            for li, L in enumerate(self.layers):
                h = self._layer_small(li, L, h, meta, kv)
            return ops.rmsnorm(h, self.final_norm, self.cfg.eps)[0]
        residual = None
        for li, L in enumerate(self.layers):
            x, residual = self._layer(li, L, x, residual, meta, kv, sk)
        return self._final_norm(x, residual)

    # Small decode batches (the interactive case): the residual stream h is the
    # only activation between layers.  The o / down projections stream their weights without split-K
    # (16-row tiles fill the chip at M <= 16) and add the residual in their epilogue, so h leaves them
    # complete; the qkv / gate_up projections read h as X and apply the RMSNorm as a per-row scale in
    # their epilogue (gains folded into their weights).  The two slab-summing RMSNorm launches per
    # layer are gone.  Switch: ``small_norm_fused`` (benchmarks/decode_ab.py A/B).  Measured SLOWER
    # (B=1 3.88 vs 3.65 ms/token, B=8 4.25 vs 3.81 ms/step, profiles/decode_small_r5.md): the whole-K
    # o / down tiles launch only N/16 workgroups, one per CU, and lose the split-K latency hiding
    # that the two norm launches cost less than -- so it is off by default.
    SMALL_FUSED_MAX_M = 16
    STREAM_CFG_RES16 = 32  # stream_gemm.hip cfg 32: BN 16, whole K
    small_norm_fused = False

    def _layer_small(self, li: int, L: DecoderLayer, h, meta: AttnMeta, kv: KVCache):
        cfg, D = self.cfg, self.cfg.head_dim
        T = h.shape[0]
        c, s = self._stream_choice("qkv", T, L.qkv_w.shape[0], L.qkv_w.shape[1])
        pg = self.proj_group
        qkv = ops.stream_gemm(h, L.qkv_w, splits=s, cfg=c, nt=True, norm_eps=cfg.eps, w_group=pg.get("qkv", 1))
        q = ops.rope_kv_write(qkv, meta.positions, self.cos_sin, kv.k[li], kv.v[li], meta.slots, self.hq, self.hkv, D)
        a = ops.paged_decode(q, kv.k[li], kv.v[li], meta.block_tables, meta.ctx_lens, meta.part_size,
                             meta.workspace, order=meta.order)
        h1 = ops.stream_gemm(a.view(T, self.hq * D), L.o_w, residual=h, cfg=self.STREAM_CFG_RES16, nt=True,
                             w_group=pg.get("o", 1))
        gc, _ = self._stream_choice("gate_up", T, L.gate_up_w.shape[0], L.gate_up_w.shape[1])
        act = ops.stream_gemm(h1, L.gate_up_w, epilogue=ops.EPI_SWIGLU8, cfg=gc, nt=True, norm_eps=cfg.eps,
                              w_group=pg.get("gate_up", 1))
        return ops.stream_gemm(act, L.down_w, residual=h1, cfg=self.STREAM_CFG_RES16, nt=True,
                               w_group=pg.get("down", 1))

    # Small decode batches: the paged attention is a chain of dependent memory round trips on a few
    # dozen CUs (~15 us per layer at batch 1 while HBM idles).  ``l3_warm_mb`` > 0 appends
    # ``l3_warm_blocks`` workgroups to that launch which read the first MB of the layer's o and
    # gate_up weights into the Infinity Cache, so those projections stream part of their weights
    # on-die.  A/B: benchmarks/decode_ab.py arms warm*.
    L3_WARM_MAX_M = 16
    l3_warm_mb = 0
    l3_warm_blocks = 192

    def _warm(self, L: DecoderLayer, T: int, ref):
        if not self.l3_warm_mb or T > self.L3_WARM_MAX_M or not ref.is_cuda:
            return None
        budget = int(self.l3_warm_mb * 2 ** 20) & ~15
        ob = L.o_w.numel() * L.o_w.element_size()
        ranges = [(L.o_w, min(ob, budget))]
        if budget > ob:
            ranges.append((L.gate_up_w, min(budget - ob, L.gate_up_w.numel() * L.gate_up_w.element_size()) & ~15))
        return ranges, self.l3_warm_blocks

    def _final_norm(self, x, residual):
        if x is None:  # the residual stream holds the last layer's output
            return ops.rmsnorm(residual, self.final_norm, self.cfg.eps)[0]
        return self._norm(x, self.final_norm, residual)[0]

    def _norm(self, x, w, residual):
        """RMSNorm(x + residual) -> (normed, new residual); x may be a ``_Partial`` whose TP
        all-reduce runs inside the same launch (``CustomAllReduce.all_reduce_rmsnorm``)."""
        if isinstance(x, _Partial):
            self.ar_counts["ipc_fused_norm"] += 1
            return self.custom_ar.all_reduce_rmsnorm(x.t, residual, w, self.cfg.eps)
        return ops.rmsnorm(x, w, self.cfg.eps, residual=residual)

    # TP decode all-reduce sites fused with their consumer RMSNorm; off: the
    # separate slab_reduce / all-reduce / rmsnorm launches (A/B and the bit-exactness test)
    tp_fused_norm = True

    def _tp_partial(self, x, cols: int):
        """A row-parallel projection's output under TP: a ``_Partial`` when the fused all-reduce +
        norm can take it, else the all-reduced bf16 tensor."""
        ar = self.custom_ar
        if self.tp_fused_norm and ar is not None and x.is_cuda and ar.norm_eligible(x, cols):
            return _Partial(x)
        if x.dtype == torch.float32 and x.dim() == 3:
            x = ops.slab_reduce(x)
        return self._all_reduce(x)

    def _layer(self, li: int, L: DecoderLayer, x, residual, meta: AttnMeta, kv: KVCache, sk: bool):
        """One decoder layer: (layer input, residual stream) -> (next layer input, residual stream)."""
        cfg, D, T = self.cfg, self.cfg.head_dim, meta.positions.numel()  # x may be [S, T, H] split-K slabs
        slabs_ok = self.tp_size == 1  # under TP the partial sums go through the all-reduce as bf16
        # prefill (TP 1): the o / down GEMMs add the residual in their epilogue (gemm256 RES, rounded
        # like the separate bf16 add), so the RMSNorms read and write one tensor instead of two each;
        # x is None then: the residual stream already holds the layer input
        fuse = not sk and self.tp_size == 1 and (x if x is not None else residual).is_cuda
        if x is None:
            h, _ = ops.rmsnorm(residual, L.attn_norm, cfg.eps)
        elif residual is None:
            h, _ = ops.rmsnorm(x, L.attn_norm, cfg.eps)
            residual = x
        else:
            h, residual = self._norm(x, L.attn_norm, residual)
        qkv = self._proj(h, L.qkv_w, sk, name="qkv")
        if (not meta.decode and not meta.n_decode and qkv.is_cuda and qkv.dtype == torch.bfloat16 and qkv.dim() == 2
                and ops.kernels.flash_rope_ok(D, kv.block_size)):
            # prefill: the RoPE/KV-write kernel writes only K / V; the attention rotates Q on load
            # straight from the projection (a [T, Hq*D] write and read less per layer)
            ops.rope_kv_write(qkv, meta.positions, self.cos_sin, kv.k[li], kv.v[li], meta.slots, self.hq, self.hkv, D,
                              write_q=False)
            q = qkv[:, :self.hq * D].view(T, self.hq, D)
            a = ops.flash_attention_paged(q, kv.k[li], kv.v[li], meta.block_tables, meta.cu_q, meta.ctx_lens,
                                          meta.max_q, causal=True, rope=(meta.positions, self.cos_sin))
            return self._layer_tail(L, a, residual, sk, fuse, slabs_ok, T, D)
        q = ops.rope_kv_write(qkv, meta.positions, self.cos_sin, kv.k[li], kv.v[li], meta.slots, self.hq, self.hkv, D)
        if meta.decode:
            a = ops.paged_decode(q, kv.k[li], kv.v[li], meta.block_tables, meta.ctx_lens, meta.part_size,
                                 meta.workspace, order=meta.order, warm=self._warm(L, T, q))
        elif meta.n_decode:
            a = self._mixed_attention(q, kv, li, meta)
        else:
            a = ops.flash_attention_paged(q, kv.k[li], kv.v[li], meta.block_tables, meta.cu_q, meta.ctx_lens,
                                          meta.max_q, causal=True)
        return self._layer_tail(L, a, residual, sk, fuse, slabs_ok, T, D)

    def _layer_tail(self, L, a, residual, sk, fuse, slabs_ok, T, D):
        """o projection, MLP norm, gate_up (+SwiGLU), down: -> (next layer input, residual stream)."""
        cfg = self.cfg
        if fuse:
            residual = ops.gemm_bt(a.view(T, self.hq * D), L.o_w, residual=residual, shuffled=self.frag,
                                   b_group=self.proj_group.get("o", 1))
            h, _ = ops.rmsnorm(residual, L.mlp_norm, cfg.eps)
        elif sk and self.tp_size > 1:
            # TP decode: the o partial (split-K slabs) meets its all-reduce inside the MLP norm's launch
            o = self._tp_partial(self._proj(a.view(T, self.hq * D), L.o_w, sk, True, name="o"), cfg.hidden)
            h, residual = self._norm(o, L.mlp_norm, residual)
        else:
            o = self._all_reduce(self._proj(a.view(T, self.hq * D), L.o_w, sk, slabs_ok, name="o"))
            h, residual = ops.rmsnorm(o, L.mlp_norm, cfg.eps, residual=residual)
        # SwiGLU in the GEMM epilogue (8-row [gate | up] groups) on the GPU
        epi = ops.EPI_SWIGLU8 if (self.interleaved_mlp and h.is_cuda) else ops.EPI_NONE
        act = self._proj(h, L.gate_up_w, sk, name="gate_up", epilogue=epi)
        if h.is_cuda and epi == ops.EPI_NONE:
            act = ops.silu_mul(act)
        if fuse:
            return None, ops.gemm_bt(act, L.down_w, residual=residual, shuffled=self.frag,
                                     b_group=self.proj_group.get("down", 1))
        if sk and self.tp_size > 1:  # reduced inside the next layer's (or the final) norm launch
            return self._tp_partial(self._proj(act, L.down_w, sk, True, name="down"), cfg.hidden), residual
        x = self._all_reduce(self._proj(act, L.down_w, sk, slabs_ok, name="down"))
        return x, residual

    @staticmethod
    def _mixed_attention(q, kv: KVCache, li: int, meta: AttnMeta) -> torch.Tensor:
        """Prefill rows through flash attention, decode rows through the split-K paged decode kernel
        (flash's 64-query tiles would be 1/64 full for them and re-read the KV per query head); both
        write disjoint row ranges of one output, so the projections around stay single GEMMs."""
        Tp = q.shape[0] - meta.n_decode
        if not q.is_cuda:
            parts = []
            if Tp:
                parts.append(ops.flash_attention_paged(q[:Tp], kv.k[li], kv.v[li], meta.block_tables, meta.cu_q,
                                                       meta.ctx_lens, meta.max_q, causal=True))
            parts.append(ops.paged_decode(q[Tp:], kv.k[li], kv.v[li], meta.dec_block_tables, meta.dec_ctx_lens,
                                          meta.part_size, meta.workspace))
            return torch.cat(parts)
        a = torch.empty_like(q)
        if Tp:
            ops.flash_attention_paged(q[:Tp], kv.k[li], kv.v[li], meta.block_tables, meta.cu_q, meta.ctx_lens,
                                      meta.max_q, causal=True, out=a[:Tp])
        ops.paged_decode(q[Tp:], kv.k[li], kv.v[li], meta.dec_block_tables, meta.dec_ctx_lens, meta.part_size,
                         meta.workspace, out=a[Tp:], order=meta.order)
        return a

    def logits(self, h: torch.Tensor) -> torch.Tensor:
        """[n, H] -> [n, V] logits (bf16; the sampler reads bf16 or fp32).  Up to 256 rows (decode
        steps, prefill last tokens) stream the fragment-layout LM head through ``stream_gemm``;
        larger batches run the MFMA GEMM on the same copy.  Vocab-parallel: [n, padded slice] with
        the first ``vocab_local`` columns valid (tokens ``vocab_start`` ...)."""
        if not h.is_cuda:
            return ops.linear(h, self.lm_head)
        return self._proj(h, self.lm_head, h.shape[0] <= self.STREAM_MAX_M, False, name="lm_head")
