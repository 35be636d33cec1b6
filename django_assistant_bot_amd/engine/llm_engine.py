"""Continuous-batching generation engine for the Llama decoder (paged KV cache, HIP graphs).

Reference behaviour replaced: ``TransformersProvider.get_response`` (ai/providers/transformers.py:35-94)
runs ``model.generate`` once per HTTP request (batch 1, fp16, top_k=50 / top_p=0.95 sampling, no
request batching across callers).  Here every concurrent request shares one batch:

  * admission / prefill: prompts are admitted while KV blocks last (native ``KVBlockManager``, with
    content-hashed prefix reuse), prompt tokens are packed into chunks of ``max_prefill_tokens``
    (long prompts are split across steps), the last prompt position is sampled;
  * decode: all running sequences advance one token per step; the step (forward + LM head + the
    sampling kernel) is replayed from a HIP graph captured per batch-size bucket, so the ~400 kernel
    launches of a decode step cost one graph launch;
  * preemption: if the pool runs dry while decoding, the youngest sequence is freed and re-queued
    (recompute), so admission can be optimistic.

Sampling parity with HF: temperature -> top-k -> top-p -> multinomial (``sample_tokens`` kernel);
``max_new_tokens`` bounds the completion (the reference's ``max_length`` counted the prompt too,
SURVEY.md 7.5; pass ``max_length`` for that behaviour).
"""
from __future__ import annotations

import itertools
import math
import os
import time
from collections import deque
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import ops
from ..models import AttnMeta, KVCache, LlamaModel, decoder_config, random_decoder_weights
from ..models.configs import DecoderConfig
from ..ops._lib import native
from ..utils import trace
from .tokenizer import Tokenizer


@dataclass
class SamplingParams:
    max_new_tokens: int = 1024
    temperature: float = 1.0
    top_k: int = 50
    top_p: float = 0.95
    ignore_eos: bool = False
    max_length: int | None = None  # HF-style cap on prompt + completion
    seed: int | None = None
    stop_token_ids: tuple = ()
    do_sample: bool = True
    timeout_s: float | None = None  # per-request deadline from arrival: finish_reason "timeout"
    json_mode: bool = False  # constrain the output to one JSON object (engine/json_constraint.py)
    json_schema: dict | str | None = None  # ... to a JSON Schema (engine/json_schema.py; implies json_mode)


@dataclass
class GenerationOutput:
    request_id: int
    prompt_ids: list
    token_ids: list
    text: str
    finish_reason: str
    usage: dict
    timings: dict


@dataclass
class _Req:
    rid: int
    prompt: list
    params: SamplingParams
    arrival: float
    out: list = field(default_factory=list)
    computed: int = 0  # prompt tokens whose KV is in the cache
    admitted: bool = False
    first_token_t: float = 0.0
    finish_t: float = 0.0
    finish_reason: str = ""
    rng_base: int = 0
    prefill_s: float = 0.0
    preempted: int = 0
    matcher: object = None  # native JsonMatcher of a json_mode request

    @property
    def seq(self):
        return self.rid

    def full_prompt(self):
        return self.prompt + self.out if self.preempted else self.prompt




def _bucket_sizes(max_batch):
    b = [1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192, 224, 256, 320, 384, 448, 512]
    return [x for x in b if x < max_batch] + [max_batch]


class LLMEngine:
    def __init__(self, model: str | DecoderConfig = "llama-3-8b", device=None, weights: dict | None = None,
                 checkpoint: str | None = None, seed: int = 0, max_batch: int = 256, block_size: int = 64,
                 max_model_len: int | None = None, kv_cache_gb: float | None = None, num_blocks: int | None = None,
                 max_prefill_tokens: int = 16384, use_graphs: bool = True, prefix_cache: bool = True,
                 tp_group=None, tp_size: int = 1, tp_rank: int = 0, interleaved_mlp: bool = True,
                 part_size: int = 512, kv_memory_fraction: float = 0.85, mixed_prefill_tokens: int = 0,
                 pipeline_decode: bool = True, shared_model: LlamaModel | None = None):
        """``shared_model``: serve with another engine's ``LlamaModel`` (one copy of the weights, a
        KV pool / scheduler / HIP graphs of this engine's own; e.g. two engines on two streams whose
        prefill and decode phases overlap: bench.py --mode overlap)."""
        self.cfg = decoder_config(model) if isinstance(model, str) else model
        cfg = self.cfg
        if checkpoint is None and weights is None and shared_model is None:
            from ..models.configs import checkpoint_dir

            checkpoint = checkpoint_dir(model)  # a local HF directory given as the model name
        self.device = torch.device(device if device is not None else ("cuda" if torch.cuda.is_available() else "cpu"))
        self.is_gpu = self.device.type == "cuda"
        self.tp_group, self.tp_size, self.tp_rank = tp_group, tp_size, tp_rank
        own_weights = weights is None  # a dict built here may be consumed while it is converted
        if shared_model is not None:
            weights = {}
        elif weights is None:
            if checkpoint:
                from ..models import load_decoder_checkpoint

                weights = load_decoder_checkpoint(checkpoint, cfg, tp_rank=tp_rank, tp_size=tp_size,
                                                  interleave_mlp=interleaved_mlp)
            else:
                weights = random_decoder_weights(cfg, self.device, seed=seed, tp_rank=tp_rank, tp_size=tp_size,
                                                 interleave_mlp=interleaved_mlp)
        if shared_model is not None:
            self.model = shared_model
        else:
            self.model = LlamaModel(cfg, weights, self.device, tp_group=tp_group, tp_size=tp_size,
                                    interleaved_mlp=interleaved_mlp, consume=own_weights, tp_rank=tp_rank)
        del weights
        if self.is_gpu and shared_model is None:
            # the caller's weight dict held the row-major originals while the model converted them
            # to the fragment layout: return those blocks to the device before the KV pool is sized
            # from the free memory (cached blocks are not "free")
            torch.cuda.empty_cache()
        if tp_size > 1 and self.is_gpu and shared_model is None:
            from ..parallel.custom_allreduce import maybe_create

            self.model.custom_ar = maybe_create(tp_group, self.device, tp_size)
        self.tokenizer = Tokenizer.for_decoder(cfg, checkpoint)
        self.max_batch = max_batch
        self.block_size = block_size
        self.max_model_len = min(max_model_len or cfg.max_position, cfg.max_position)
        self.max_blocks_per_seq = math.ceil(self.max_model_len / block_size)
        self.max_prefill_tokens = max_prefill_tokens
        self.mixed_prefill_tokens = mixed_prefill_tokens
        self.part_size = part_size
        # Key partition of the split-K decode attention per step size: partitions of 2048 keys (one
        # per sequence at RAG context lengths) stream 12 % faster than 512 at batch 128 (fewer
        # combines, longer streams per workgroup: benchmarks/kernel_bench.py decode), but small
        # batches need the finer split to give every CU work.
        self.long_part_size = max(part_size, 2048)
        hkv = cfg.kv_heads // tp_size
        per_block = KVCache.bytes_per_block(cfg.layers, hkv, block_size, cfg.head_dim)
        if num_blocks is None:
            if kv_cache_gb:
                num_blocks = int(kv_cache_gb * (1 << 30) // per_block)
            elif self.is_gpu:
                free, _ = torch.cuda.mem_get_info(self.device)
                num_blocks = int(free * kv_memory_fraction // per_block)
            else:
                num_blocks = 4 * self.max_blocks_per_seq
            num_blocks = max(2, min(num_blocks, max_batch * self.max_blocks_per_seq + 8))
        self.kv = KVCache(cfg.layers, num_blocks, hkv, block_size, cfg.head_dim, self.device)
        self.blocks = native().KVBlockManager(num_blocks, block_size, prefix_cache)
        self._prefix_cache = prefix_cache
        self.seed = seed
        self.waiting: deque[_Req] = deque()
        self.prefilling: list[_Req] = []
        self.running: list[_Req] = []
        self.finished: dict[int, _Req] = {}
        self._ids = itertools.count()
        self.stats = {"prefill_tokens": 0, "decode_tokens": 0, "decode_steps": 0, "prefill_steps": 0,
                      "preemptions": 0, "graph_replays": 0, "mixed_steps": 0}
        # decode static buffers (graph inputs / outputs)
        self.use_graphs = use_graphs and self.is_gpu
        dev = self.device
        mb = max_batch
        self._d_ids = torch.zeros(mb, dtype=torch.int32, device=dev)
        self._d_pos = torch.zeros(mb, dtype=torch.int32, device=dev)
        self._d_slots = torch.full((mb,), -1, dtype=torch.int64, device=dev)
        self._d_ctx = torch.ones(mb, dtype=torch.int32, device=dev)
        self._d_bt = torch.zeros((mb, self.max_blocks_per_seq), dtype=torch.int32, device=dev)
        self._d_temp = torch.ones(mb, dtype=torch.float32, device=dev)
        self._d_topk = torch.full((mb,), 50, dtype=torch.int32, device=dev)
        self._d_topp = torch.ones(mb, dtype=torch.float32, device=dev)
        self._d_cnt = torch.zeros(mb, dtype=torch.int64, device=dev)
        self._d_tokens = torch.zeros(mb, dtype=torch.int32, device=dev)
        self._d_order = torch.arange(mb, dtype=torch.int32, device=dev)  # decode attention dispatch order
        pin = self.is_gpu
        mk = lambda *a, **k: torch.zeros(*a, **k, pin_memory=pin)  # noqa: E731
        self._h_ids = mk(mb, dtype=torch.int32)
        self._h_pos = mk(mb, dtype=torch.int32)
        self._h_slots = mk(mb, dtype=torch.int64)
        self._h_ctx = mk(mb, dtype=torch.int32)
        self._h_bt = mk((mb, self.max_blocks_per_seq), dtype=torch.int32)
        self._h_temp = mk(mb, dtype=torch.float32)
        self._h_topk = mk(mb, dtype=torch.int32)
        self._h_topp = mk(mb, dtype=torch.float32)
        self._h_cnt = mk(mb, dtype=torch.int64)
        self._h_tokens = mk(mb, dtype=torch.int32)
        self._h_order = mk(mb, dtype=torch.int32)
        # pipelined decode (``_step_pipelined``): step t+1 is launched before step t's tokens are read,
        # its input ids copied on the device from step t's sampled tokens, so the host's per-step
        # bookkeeping overlaps the GPU instead of idling it.  Two alternating host buffer sets: the
        # H2D copies of step t may still be pending while step t+1's are filled.
        self.pipeline_decode = bool(pipeline_decode) and tp_size == 1
        self._h_alt = {k: mk(*(getattr(self, k).shape,), dtype=getattr(self, k).dtype)
                       for k in ("_h_ids", "_h_pos", "_h_slots", "_h_ctx", "_h_bt", "_h_temp", "_h_topk", "_h_topp",
                                 "_h_cnt", "_h_tokens", "_h_order")}
        self._inflight = None  # launched decode step whose tokens are not consumed yet
        self._d_mask = None  # JSON-constrained decoding buffers (allocated on first use)
        self._masked = False
        # launched prefill chunk whose sampled first tokens are not read back yet (GPU): the next
        # chunk is launched before they are, so consecutive chunks run back to back
        self._pending_prefill = None
        max_parts = math.ceil(self.max_model_len / part_size)
        self._workspace = ops.DecodeWorkspace(mb, cfg.heads // tp_size, cfg.head_dim, max_parts, dev) if self.is_gpu \
            else None
        self._sample_ws = ops.kernels.sample_workspace(mb, cfg.vocab_size, dev) if self.is_gpu else None
        # vocab-parallel LM head (TP): the decode graph ends with this rank's sampling candidates;
        # the all-gather and the merge that draws the token run after the replay (_vp_merge)
        self.vp = bool(getattr(self.model, "vocab_parallel", False))
        self._vp_cand = None
        if self.vp and self.is_gpu:
            ncl = ops.kernels.sample_candidates_per_row(self.model.vocab_local)
            self._vp_cand = torch.zeros((2, mb, ncl), dtype=torch.int32, device=dev)
        self._graphs: dict = {}
        self._buckets = _bucket_sizes(max_batch)
        self._graph_pool = None
        # GPU spans of the engine phases (HIP events, read where the host syncs anyway) -> stats
        self.timer = trace.GpuTimer(enabled=self.is_gpu)
        # test hook: called at the start of every step (fault injection, e.g. raise a HIP error)
        self.fault_hook = None
        # deadlines are checked by step() unless a TP leader drives them explicitly (wall clocks of
        # the ranks differ; every rank must drop a request at the same step)
        self.auto_expire = True

    # ------------------------------------------------------------------ public API
    def add_request(self, prompt_ids: list, params: SamplingParams | None = None, request_id: int | None = None) -> int:
        params = params or SamplingParams()
        rid = next(self._ids) if request_id is None else request_id
        prompt = [int(t) for t in prompt_ids]
        if not prompt:
            prompt = [self.cfg.bos_id]
        if len(prompt) >= self.max_model_len:
            prompt = prompt[-(self.max_model_len - 1):]
        seed = params.seed if params.seed is not None else self.seed
        r = _Req(rid, prompt, params, time.perf_counter(), rng_base=((seed * 1000003 + rid) & 0xFFFFFFFF) << 20)
        r.matcher = self.check_params(params, matcher=True)
        if r.matcher is not None:
            self._ensure_mask_buffers()
        self.waiting.append(r)
        return rid

    def check_params(self, params: SamplingParams, matcher: bool = False):
        """Validates a request's decoding constraint (raises ``SchemaError`` for a schema the
        constrained decoder cannot compile) and, with ``matcher``, returns the request's native
        matcher (None when unconstrained).  Callers that queue requests for another rank's engine
        (``NodeLLM``) call it first, so a bad schema fails its caller, never the remote step."""
        if params.json_schema is not None and self.tokenizer.byte_exact:
            from .json_schema import automaton_for, matcher_for

            if not matcher:
                automaton_for(self.tokenizer, self.cfg.eos_ids, params.json_schema)  # cached per schema
                return None
            return matcher_for(self.tokenizer, self.cfg.eos_ids, params.json_schema)
        if params.json_mode or params.json_schema is not None:
            # (the offline hash tokenizer puts a space before every word token, so exact keys /
            # enum strings cannot be spelled: a schema degrades to plain JSON mode there; it is
            # still validated, so an unsupported schema fails the same way everywhere)
            from .json_constraint import matcher_for

            if params.json_schema is not None:
                from .json_schema import compile_schema

                compile_schema(params.json_schema)
            return matcher_for(self.tokenizer, self.cfg.eos_ids) if matcher else None
        return None

    def rejected_output(self, rid: int, prompt_ids, reason: str) -> GenerationOutput:
        """The output of a request that could not be admitted (no tokens, ``finish_reason`` =
        ``"error: ..."``): answers its caller instead of failing the step it arrived in."""
        return GenerationOutput(request_id=rid, prompt_ids=list(prompt_ids), token_ids=[], text="",
                                finish_reason=f"error: {reason}",
                                usage={"prompt_tokens": len(prompt_ids), "completion_tokens": 0,
                                       "total_tokens": len(prompt_ids)},
                                timings={"queue_s": 0.0, "ttft_s": 0.0, "total_s": 0.0, "decode_s": 0.0,
                                         "prefill_s": 0.0})

    def has_unfinished(self) -> bool:
        return bool(self.waiting or self.prefilling or self.running)

    def generate(self, prompts: list, params: SamplingParams | list | None = None) -> list[GenerationOutput]:
        """Batch generate: token-id lists or strings -> outputs in input order."""
        plist = params if isinstance(params, list) else [params or SamplingParams()] * len(prompts)
        rids = []
        for p, sp in zip(prompts, plist):
            ids = self.tokenizer.encode(p) if isinstance(p, str) else p
            rids.append(self.add_request(ids, sp))
        while self.has_unfinished():
            self.step()
        return [self.pop_output(r) for r in rids]

    def pop_output(self, rid: int) -> GenerationOutput:
        r = self.finished.pop(rid)
        n_out = len(r.out)
        return GenerationOutput(
            request_id=rid, prompt_ids=r.prompt, token_ids=list(r.out),
            text=self.tokenizer.decode(r.out), finish_reason=r.finish_reason,
            usage={"prompt_tokens": len(r.prompt), "completion_tokens": n_out, "total_tokens": len(r.prompt) + n_out},
            timings={"queue_s": max(0.0, r.first_token_t - r.arrival - r.prefill_s),
                     "ttft_s": r.first_token_t - r.arrival, "total_s": r.finish_t - r.arrival,
                     "decode_s": r.finish_t - r.first_token_t, "prefill_s": r.prefill_s},
        )

    def step(self) -> list[int]:
        """One scheduler iteration. Returns the ids finished by it.

        * nothing running: a prefill step (chunks of up to ``max_prefill_tokens``);
        * running sequences and pending prompts with ``mixed_prefill_tokens`` > 0: ONE mixed forward
          -- every running sequence decodes a token and up to ``mixed_prefill_tokens`` prompt tokens
          ride along in the same GEMMs (a decode-sized GEMM is weight-read bound, so the first few
          hundred extra rows are nearly free and the rest run at prefill efficiency), instead of
          stalling all decodes for a whole prefill step;
        * otherwise a decode step (HIP-graph replay).
        """
        done_before = set(self.finished)
        if self.fault_hook is not None:
            self.fault_hook(self)
        if self.auto_expire:
            self.expire_deadlines()
        if self._pending_prefill is not None:
            # another plain prefill chunk goes onto the GPU before the previous one's tokens are read
            chunks = self._schedule_prefill() if not self.running or self.mixed_prefill_tokens <= 0 else []
            if chunks:
                prev, self._pending_prefill = self._pending_prefill, None
                self._run_prefill(chunks)
                self._finish_prefill(prev)
                return [k for k in self.finished if k not in done_before]
            self._finish_prefill(self._pending_prefill)
            self._pending_prefill = None
        if self._inflight is not None and not self._can_pipeline():
            self._finish_inflight()
        if self._can_pipeline():
            self._step_pipelined()
        elif self.running and self.mixed_prefill_tokens > 0 and (self.waiting or self.prefilling):
            batch = self._reserve_decode()
            chunks = self._schedule_prefill(self.mixed_prefill_tokens) if batch else self._schedule_prefill()
            if chunks and batch:
                self._run_mixed(batch, chunks)
            elif chunks:
                self._run_prefill(chunks)
            elif batch:
                self._run_decode(batch)
        else:
            chunks = self._schedule_prefill()
            if chunks:
                self._run_prefill(chunks)
            elif self.running:
                batch = self._reserve_decode()
                if batch:
                    self._run_decode(batch)
        return [k for k in self.finished if k not in done_before]

    def abort(self, rid: int, reason: str = "abort") -> bool:
        """Stops a request wherever it is (queued, prefilling or decoding) and frees its KV blocks;
        its output (tokens so far) is kept under ``finish_reason=reason``."""
        if self._inflight is not None:
            self._finish_inflight()
        if self._pending_prefill is not None:
            pend, self._pending_prefill = self._pending_prefill, None
            self._finish_prefill(pend)
        for q in (self.waiting, self.prefilling, self.running):
            for r in q:
                if r.rid == rid:
                    q.remove(r)
                    if r.admitted:
                        self.blocks.free_sequence(r.seq)
                    r.finish_reason = reason
                    r.finish_t = time.perf_counter()
                    self.finished[rid] = r
                    self.stats["aborted"] = self.stats.get("aborted", 0) + 1
                    return True
        return False

    def fail_all(self) -> list[int]:
        """Drops every unfinished request (after an engine fault) and returns their ids; the block
        pool is rebuilt so nothing leaks if the fault left the bookkeeping half-updated."""
        ids = [r.rid for q in (self.waiting, self.prefilling, self.running) for r in q]
        self._inflight = None
        self._pending_prefill = None
        self.waiting.clear()
        self.prefilling.clear()
        self.running.clear()
        self.blocks = native().KVBlockManager(self.blocks.num_blocks(), self.block_size, self._prefix_cache)
        self.timer.collect()
        return ids

    def expired(self) -> list[int]:
        now = time.perf_counter()
        return [r.rid for q in (self.waiting, self.prefilling, self.running) for r in q
                if r.params.timeout_s is not None and now - r.arrival > r.params.timeout_s]

    def expire_deadlines(self) -> list[int]:
        ids = self.expired()
        for rid in ids:
            self.abort(rid, "timeout")
        return ids

    # ------------------------------------------------------------------ scheduling
    def _schedule_prefill(self, budget: int | None = None):
        budget = self.max_prefill_tokens if budget is None else budget
        chunks = []
        for r in self.prefilling:
            if budget <= 0:
                break
            total = len(r.full_prompt())
            n = min(total - r.computed, budget)
            if n > 0:
                chunks.append((r, r.computed, n))
                self.blocks.commit_prefix(r.seq, r.computed + n)
                budget -= n
        while self.waiting and budget > 0 and len(self.running) + len(self.prefilling) < self.max_batch:
            r = self.waiting[0]
            toks = r.full_prompt()
            cached = self.blocks.add_sequence(r.seq, toks, 1)
            if cached < 0:
                if not self.running and not self.prefilling:
                    raise RuntimeError("KV cache too small for a single request")
                break
            self.waiting.popleft()
            r.admitted = True
            r.computed = cached
            self.prefilling.append(r)
            n = min(len(toks) - cached, budget)
            chunks.append((r, cached, n))
            # the chunk's full blocks enter the prefix cache as it is scheduled: a later request of
            # the SAME step that shares them (a common system prompt) starts after them.  Every chunk
            # scheduled here runs in one forward whose per-layer K / V write covers all of its tokens
            # before that layer's attention reads any block, so the sharer reads them in time.
            self.blocks.commit_prefix(r.seq, cached + n)
            budget -= n
        return chunks

    def _build_block_tables(self, seqs, out_host):
        self.blocks.block_table_into(seqs, self.max_blocks_per_seq, out_host.data_ptr())

    def _run_prefill(self, chunks):
        t0 = time.perf_counter()
        B = len(chunks)
        T = sum(n for _, _, n in chunks)
        ids = np.empty(T, dtype=np.int32)
        pos = np.empty(T, dtype=np.int32)
        slots = torch.empty(T, dtype=torch.int64)
        cu = np.zeros(B + 1, dtype=np.int32)
        ctx = np.empty(B, dtype=np.int32)
        o = 0
        for i, (r, s, n) in enumerate(chunks):
            toks = r.full_prompt()
            ids[o:o + n] = toks[s:s + n]
            pos[o:o + n] = np.arange(s, s + n, dtype=np.int32)
            self.blocks.slot_mapping_into(r.seq, s, n, slots.data_ptr() + 8 * o)
            o += n
            cu[i + 1] = o
            ctx[i] = s + n
        bt = torch.zeros((B, self.max_blocks_per_seq), dtype=torch.int32)
        self._build_block_tables([r.seq for r, _, _ in chunks], bt)
        to = self._h2d
        meta = AttnMeta(decode=False, positions=to(pos), slots=to(slots), block_tables=to(bt), ctx_lens=to(ctx),
                        cu_q=to(cu), max_q=max(n for _, _, n in chunks))
        with self.timer.phase("prefill"):
            hidden = self.model.forward(to(ids), meta, self.kv)
        last_rows = [i for i, (r, s, n) in enumerate(chunks) if s + n == len(r.full_prompt())]
        self.stats["prefill_tokens"] += T
        self.stats["prefill_steps"] += 1
        reqs, toks = [], []
        if last_rows:
            sel = self._h2d(torch.as_tensor([int(cu[i + 1]) - 1 for i in last_rows], dtype=torch.long))
            logits = self.model.logits(hidden.index_select(0, sel))
            reqs = [chunks[i][0] for i in last_rows]
            toks = self._sample(logits, reqs, to_host=not self.is_gpu)
        for r, s, n in chunks:
            r.computed = s + n
            # register the chunk's full blocks in the prefix cache at launch: the hashes depend only
            # on the tokens, and any forward that reuses them is enqueued behind this one on the
            # stream, so a request admitted while this chunk's read-back is deferred already hits
            # the shared prefix (e.g. the system prompt) instead of recomputing it
            self.blocks.commit_prefix(r.seq, s + n)
        pend = (chunks, reqs, toks, t0)
        self._tp_fault_enqueue()
        if self.is_gpu:
            self._pending_prefill = pend  # read back after the next launch (step)
        else:
            self._finish_prefill(pend)

    def _finish_prefill(self, pend):
        """Reads a launched prefill chunk's sampled first tokens (device -> host) and moves the
        sequences whose prompt it completed to the running set."""
        chunks, reqs, toks, t0 = pend
        if torch.is_tensor(toks):
            toks = toks.cpu().tolist()
            self._tp_fault_check()  # synchronised: the error word copied behind the chunk is current
        self._collect_gpu_times(block=bool(reqs))
        now = time.perf_counter()
        for r, s, n in chunks:
            r.prefill_s += now - t0
        if reqs:
            for r, t in zip(reqs, toks):
                self.blocks.commit_prefix(r.seq, len(r.full_prompt()))
                self.prefilling.remove(r)
                r.first_token_t = r.first_token_t or now
                r.preempted = 0
                self.running.append(r)
                self._accept_token(r, int(t), now)

    def _h2d(self, a):
        """Host array -> device tensor on the current stream, from pinned memory on the GPU so the
        copy is asynchronous (a pageable copy blocks the host until the stream reaches it, so the
        next prefill chunk could not be enqueued behind the running one)."""
        t = torch.as_tensor(a)
        if not self.is_gpu:
            return t
        return t.pin_memory().to(self.device, non_blocking=True)

    def _run_mixed(self, batch: list, chunks):
        """Prefill chunks + one decode token per running sequence in one forward (see ``step``)."""
        t0 = time.perf_counter()
        dev = self.device
        B = len(batch)
        P = len(chunks)
        Tp = sum(n for _, _, n in chunks)
        # pad the decode rows (slot -1, one key of block 0, output ignored) so the GEMM M is a
        # multiple of 64: full MFMA tiles in the prefill GEMMs
        Bp = B + (-(Tp + B)) % 64 if self.is_gpu else B
        Bp = min(Bp, self.max_batch)
        T = Tp + Bp
        ids = torch.empty(T, dtype=torch.int32, pin_memory=self.is_gpu)
        pos = torch.empty(T, dtype=torch.int32, pin_memory=self.is_gpu)
        slots = torch.empty(T, dtype=torch.int64, pin_memory=self.is_gpu)
        cu = np.zeros(P + 1, dtype=np.int32)
        ctx = np.empty(P, dtype=np.int32)
        ids_np, pos_np = ids.numpy(), pos.numpy()
        o = 0
        for i, (r, s, n) in enumerate(chunks):
            toks = r.full_prompt()
            ids_np[o:o + n] = toks[s:s + n]
            pos_np[o:o + n] = np.arange(s, s + n, dtype=np.int32)
            self.blocks.slot_mapping_into(r.seq, s, n, slots.data_ptr() + 8 * o)
            o += n
            cu[i + 1] = o
            ctx[i] = s + n
        if Bp > B:
            self._h_ids[B:Bp] = 0
            self._h_pos[B:Bp] = 0
            self._h_slots[B:Bp] = -1
            self._h_ctx[B:Bp] = 1
            self._h_bt[B:Bp] = 0
        ids[Tp:] = self._h_ids[:Bp]
        pos[Tp:] = self._h_pos[:Bp]
        slots[Tp:] = self._h_slots[:Bp]
        bt = torch.zeros((P, self.max_blocks_per_seq), dtype=torch.int32)
        self._build_block_tables([r.seq for r, _, _ in chunks], bt)
        to = lambda a: torch.as_tensor(a).to(dev, non_blocking=True)  # noqa: E731
        self._d_ctx[:Bp].copy_(self._h_ctx[:Bp], non_blocking=True)
        self._d_bt[:Bp].copy_(self._h_bt[:Bp], non_blocking=True)
        order = None
        if self.is_gpu:  # longest first: the decode attention stops at the longest context's partitions
            self._fill_order(Bp)
            self._d_order[:Bp].copy_(self._h_order[:Bp], non_blocking=True)
            order = self._d_order[:Bp]
        meta = AttnMeta(decode=False, positions=to(pos), slots=to(slots), block_tables=to(bt), ctx_lens=to(ctx),
                        cu_q=to(cu), max_q=max(n for _, _, n in chunks), workspace=self._workspace,
                        part_size=self._decode_part(Bp), n_decode=Bp, dec_block_tables=self._d_bt[:Bp],
                        dec_ctx_lens=self._d_ctx[:Bp], order=order)
        with self.timer.phase("mixed"):
            hidden = self.model.forward(to(ids), meta, self.kv)
        last_rows = [i for i, (r, s, n) in enumerate(chunks) if s + n == len(r.full_prompt())]
        sel = [int(cu[i + 1]) - 1 for i in last_rows] + list(range(Tp, Tp + B))
        sel_d = torch.as_tensor(sel, dtype=torch.long).to(dev, non_blocking=True)
        logits = self.model.logits(hidden.index_select(0, sel_d))
        preqs = [chunks[i][0] for i in last_rows]
        self._tp_fault_enqueue()
        toks = self._sample(logits, preqs + batch)
        self._tp_fault_check()
        self._collect_gpu_times()
        now = time.perf_counter()
        self.stats["prefill_tokens"] += Tp
        self.stats["decode_tokens"] += B
        self.stats["decode_steps"] += 1
        self.stats["mixed_steps"] += 1
        for r, s, n in chunks:
            r.computed = s + n
            r.prefill_s += now - t0
        for r, t in zip(batch, toks[len(preqs):]):
            self._accept_token(r, int(t), now)
        for r, t in zip(preqs, toks[:len(preqs)]):
            self.blocks.commit_prefix(r.seq, len(r.full_prompt()))
            self.prefilling.remove(r)
            r.first_token_t = r.first_token_t or now
            r.preempted = 0
            self.running.append(r)
            self._accept_token(r, int(t), now)

    def _collect_gpu_times(self, block: bool = True):
        for name, ms in self.timer.collect(block).items():
            key = f"gpu_{name}_ms"
            self.stats[key] = self.stats.get(key, 0.0) + ms

    # ------------------------------------------------------------------ JSON-constrained rows
    def _ensure_mask_buffers(self) -> None:
        if getattr(self, "_d_mask", None) is not None:
            return
        W = -(-self.cfg.vocab_size // 32)
        mb = self.max_batch
        pin = self.is_gpu
        # two pinned host sets, alternated: a launched prefill chunk's mask copy may still be queued
        # behind its forward when the next chunk fills masks (each set is reused only after the copy
        # issued from it two calls ago has run)
        self._h_masks = [(torch.zeros((mb, W), dtype=torch.int32, pin_memory=pin),
                          torch.zeros(mb, dtype=torch.int32, pin_memory=pin)) for _ in range(2)]
        self._mask_events = [None, None]
        self._mask_turn = 0
        self._d_mask = torch.zeros((mb, W), dtype=torch.int32, device=self.device)
        self._d_mflag = torch.zeros(mb, dtype=torch.int32, device=self.device)

    def _budget(self, r: _Req) -> int:
        """Tokens ``r`` may still generate, the one being sampled included."""
        n, p = len(r.out), r.params
        left = min(p.max_new_tokens - n, self.max_model_len - len(r.prompt) - n)
        if p.max_length is not None:
            left = min(left, p.max_length - len(r.prompt) - n)
        return max(left, 1)

    def _fill_masks(self, reqs, n_rows: int) -> bool:
        """Host masks + row flags of the constrained rows among ``reqs`` (rows past them unflagged)
        and their H2D copies.  -> whether any row is constrained."""
        if not any(r.matcher is not None for r in reqs):
            return False
        t = self._mask_turn
        self._mask_turn ^= 1
        if self._mask_events[t] is not None:
            self._mask_events[t].synchronize()
        h_mask, h_flag = self._h_masks[t]
        h_flag[:n_rows] = 0
        row_bytes = h_mask.shape[1] * 4
        base = h_mask.data_ptr()
        for i, r in enumerate(reqs):
            if r.matcher is not None:
                r.matcher.fill_mask(self._budget(r), base + i * row_bytes)
                h_flag[i] = 1
        self._d_mask[:n_rows].copy_(h_mask[:n_rows], non_blocking=True)
        self._d_mflag[:n_rows].copy_(h_flag[:n_rows], non_blocking=True)
        if self.is_gpu:
            ev = torch.cuda.Event()
            ev.record()
            self._mask_events[t] = ev
        return True

    def _mask(self, logits, rows: int):
        m = self.model
        ops.mask_logits(logits, self._d_mask[:rows], self._d_mflag[:rows], vocab=getattr(m, "vocab_local", None),
                        word_offset=getattr(m, "vocab_start", 0) // 32)

    def _vp_merge(self, cand, temp, topk, topp, cnt, out=None):
        """Vocab-parallel draw: all-gather every TP rank's candidates [2, rows, n] and merge them
        (``ops.sample_merge``); every rank gets the same tokens from the same counters."""
        import torch.distributed as dist

        src = cand.contiguous()
        if dist.get_backend(self.tp_group) != "nccl":  # gloo rehearsal of the TP group on one GPU
            src = src.cpu()
        parts = [torch.empty_like(src) for _ in range(self.tp_size)]
        dist.all_gather(parts, src, group=self.tp_group)
        allc = torch.stack(parts, 2).to(self.device)  # [2, rows, tp, n]
        allc = allc.reshape(2, allc.shape[1], -1).contiguous()
        return ops.sample_merge(allc, temp, topk, topp, self.seed, cnt, self.cfg.vocab_size, out=out)

    def _sample(self, logits, reqs, to_host: bool = True):
        n = len(reqs)
        if self._fill_masks(reqs, n):
            self._mask(logits, n)
        temps = torch.tensor([r.params.temperature if r.params.do_sample else 0.0 for r in reqs], dtype=torch.float32)
        topk = torch.tensor([r.params.top_k for r in reqs], dtype=torch.int32)
        topp = torch.tensor([r.params.top_p for r in reqs], dtype=torch.float32)
        cnt = torch.tensor([r.rng_base + len(r.out) for r in reqs], dtype=torch.int64)
        if self.is_gpu:
            fast = all((0 < r.params.top_k <= ops.kernels.SAMPLE_FAST_MAX_K) or not r.params.do_sample
                       or r.params.temperature <= 0 for r in reqs)
            h = self._h2d
            if self.vp and fast:
                cand = ops.sample_candidates(logits, self.model.vocab_local, self.model.vocab_start)
                toks = self._vp_merge(cand, h(temps), h(topk), h(topp), h(cnt))
            else:
                if self.vp:  # exact full-vocabulary sampling (top_k off or > 64): gather the logits
                    logits = self.model.full_logits(logits)
                toks = ops.sample_tokens(logits, h(temps), h(topk), h(topp), self.seed, h(cnt), fast=fast)
                toks = self._tp_sync_tokens(toks)
            return toks.cpu().tolist() if to_host else toks
        if self.vp:
            logits = self.model.full_logits(logits)
        g = torch.Generator().manual_seed(int(self.seed * 7919 + int(cnt[0]) if n else 0))
        return ops.sample_tokens(logits, temps, topk, topp, self.seed, cnt, generator=g).tolist()

    # ------------------------------------------------------------------ TP fault path
    def _tp_fault_enqueue(self) -> None:
        """TP on the GPU: the one-shot all-reduce's sticky error word is copied to the host behind
        the step just enqueued (no sync here)."""
        ar = getattr(self.model, "custom_ar", None)
        if ar is not None and self.is_gpu:
            ar.enqueue_error_check()

    def _tp_fault_check(self) -> None:
        """After the step's own sync: a set word means a TP peer missed an all-reduce (desynchronised
        or dead group).  The step's outputs are poisoned, so it raises ``CustomAllReduceError`` before
        any of its tokens is accepted; ``LLMWorker`` fails the in-flight requests (HTTP 500, as the
        reference's failed ``generate``: gpu_service/main.py:105-107) and turns unhealthy (/health
        503), and the launcher restarts the group."""
        ar = getattr(self.model, "custom_ar", None)
        if ar is not None and self.is_gpu:
            ar.raise_if_error()

    def _tp_sync_tokens(self, toks):
        if self.tp_size > 1:
            import torch.distributed as dist

            src = dist.get_global_rank(self.tp_group, 0) if self.tp_group is not None else 0
            dist.broadcast(toks, src=src, group=self.tp_group)
        return toks

    def _accept_token(self, r: _Req, tok: int, now: float):
        r.out.append(tok)
        p = r.params
        reason = ""
        json_done = False
        if r.matcher is not None:
            if r.matcher.advance(tok):
                json_done = r.matcher.done()
            else:  # only after a mask fallback (no grammar-valid token was left)
                self.stats["json_broken"] = self.stats.get("json_broken", 0) + 1
        if json_done:
            reason = "stop"  # the JSON object is complete
        elif not p.ignore_eos and (tok in self.cfg.eos_ids or tok in p.stop_token_ids):
            reason = "stop"
        elif len(r.out) >= p.max_new_tokens:
            reason = "length"
        elif p.max_length is not None and len(r.prompt) + len(r.out) >= p.max_length:
            reason = "length"
        elif len(r.prompt) + len(r.out) >= self.max_model_len:
            reason = "length"
        if reason:
            r.finish_reason = reason
            r.finish_t = now
            self.running.remove(r)
            self.blocks.free_sequence(r.seq)
            self.finished[r.rid] = r

    def _preempt_one(self, protect: _Req | None) -> bool:
        for victim in reversed(self.running):
            if victim is protect:
                continue
            self.running.remove(victim)
            self.blocks.free_sequence(victim.seq)
            victim.preempted = 1
            victim.computed = 0
            self.waiting.appendleft(victim)
            self.stats["preemptions"] += 1
            return True
        return False

    # ------------------------------------------------------------------ pipelined decode
    def _can_pipeline(self) -> bool:
        # constrained rows need each token on the host before the next step's mask
        return bool(self.pipeline_decode and self.running and not self.waiting and not self.prefilling
                    and not any(r.matcher is not None for r in self.running))

    def _swap_host_buffers(self) -> None:
        for k, alt in self._h_alt.items():
            cur = getattr(self, k)
            setattr(self, k, alt)
            self._h_alt[k] = cur

    def _length_done(self, r: _Req, extra: int) -> bool:
        """Whether ``r`` stops for length once ``extra`` more tokens are accepted (EOS / stop tokens
        are unknowable in advance: such a sequence decodes one wasted token, discarded)."""
        n, p = len(r.out) + extra, r.params
        return (n >= p.max_new_tokens or (p.max_length is not None and len(r.prompt) + n >= p.max_length)
                or len(r.prompt) + n >= self.max_model_len)

    def _step_pipelined(self):
        """One decode step with the next one already on the GPU: launch step t+1 (ids = step t's
        device tokens), then consume step t's tokens.  Finishes that the host can predict (length
        limits) leave the next batch before it is launched."""
        prev = self._inflight
        if prev is None:
            batch = self._reserve_decode()
            if not batch:
                return
            self._launch_decode(batch, None)
            prev = self._inflight
        nxt = [r for r in prev["batch"] if not r.finish_reason and not self._length_done(r, 1)]
        launched = False
        if nxt:
            self._swap_host_buffers()
            fail = self.blocks.prepare_decode_into(
                [r.seq for r in nxt], [r.out[-1] if r.out else 0 for r in nxt], self.max_blocks_per_seq,
                self._h_ids.data_ptr(), self._h_pos.data_ptr(), self._h_slots.data_ptr(), self._h_ctx.data_ptr(),
                self._h_bt.data_ptr())
            if fail < 0:
                pos = {id(r): i for i, r in enumerate(prev["batch"])}
                self._launch_decode(nxt, [pos[id(r)] for r in nxt], pending=1)
                launched = True
            else:  # pool dry: finish step t, the synchronous path preempts
                self._swap_host_buffers()
        cur = self._inflight if launched else None
        self._inflight = prev
        self._finish_inflight()
        self._inflight = cur

    def _launch_decode(self, batch: list, src_rows, pending: int = 0):
        """Enqueue one decode step for ``batch`` (host metadata already in the _h_* buffers).
        ``src_rows``: None -> input ids from the host buffer; else row i's input token is row
        src_rows[i] of the previous step's device tokens.  ``pending`` tokens per sequence are
        sampled but not yet appended (RNG counters count them)."""
        t0 = time.perf_counter()
        B = len(batch)
        self._h_temp[:B] = torch.tensor([r.params.temperature if r.params.do_sample else 0.0 for r in batch])
        self._h_topk[:B] = torch.tensor([r.params.top_k for r in batch], dtype=torch.int32)
        self._h_topp[:B] = torch.tensor([r.params.top_p for r in batch])
        self._h_cnt[:B] = torch.tensor([r.rng_base + len(r.out) + pending for r in batch], dtype=torch.int64)
        self._fast = all((0 < r.params.top_k <= ops.kernels.SAMPLE_FAST_MAX_K) or not r.params.do_sample
                         or r.params.temperature <= 0 for r in batch)
        Bp = next(b for b in self._buckets if b >= B) if self.use_graphs else B
        if Bp > B:
            self._h_ids[B:Bp] = 0
            self._h_pos[B:Bp] = 0
            self._h_slots[B:Bp] = -1
            self._h_ctx[B:Bp] = 1
            self._h_bt[B:Bp] = 0
            self._h_temp[B:Bp] = 0.0
            self._h_topk[B:Bp] = 1
            self._h_topp[B:Bp] = 1.0
            self._h_cnt[B:Bp] = 0
        self._fill_order(Bp)
        pairs = [(self._d_pos, self._h_pos), (self._d_slots, self._h_slots), (self._d_ctx, self._h_ctx),
                 (self._d_temp, self._h_temp), (self._d_topk, self._h_topk), (self._d_topp, self._h_topp),
                 (self._d_cnt, self._h_cnt), (self._d_bt, self._h_bt), (self._d_order, self._h_order)]
        if src_rows is None:
            pairs.append((self._d_ids, self._h_ids))
        else:
            # stream-ordered after the previous step's sampling kernel
            if src_rows == list(range(B)):
                self._d_ids[:B].copy_(self._d_tokens[:B])
            else:
                idx = torch.as_tensor(src_rows, dtype=torch.long).to(self.device, non_blocking=True)
                self._d_ids[:B].copy_(self._d_tokens.index_select(0, idx))
            if Bp > B:
                self._d_ids[B:Bp].zero_()
        for d, h in pairs:
            d[:Bp].copy_(h[:Bp], non_blocking=True)
        self._masked = False
        g = None
        if self.use_graphs:
            g = self._graphs.get((Bp, self._fast, False))
            if g is None:
                g = self._capture(Bp)
        with self.timer.phase("decode"):
            if g is not None:
                g.replay()
                self.stats["graph_replays"] += 1
            else:
                self._decode_body(Bp)
        ev = None
        if self.is_gpu:
            self._h_tokens[:Bp].copy_(self._d_tokens[:Bp], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        self._inflight = {"batch": list(batch), "Bp": Bp, "tokens": self._h_tokens, "event": ev}
        self.stats["decode_host_s"] = self.stats.get("decode_host_s", 0.0) + time.perf_counter() - t0

    def _finish_inflight(self):
        inf, self._inflight = self._inflight, None
        if inf is None:
            return
        t1 = time.perf_counter()
        if inf["event"] is not None:
            inf["event"].synchronize()
        t2 = time.perf_counter()
        self._collect_gpu_times(block=False)
        batch = inf["batch"]
        toks = inf["tokens"][:len(batch)].tolist()
        now = time.perf_counter()
        self.stats["decode_steps"] += 1
        for r, t in zip(batch, toks):
            if r.finish_reason:  # finished (EOS) or aborted while this step was in flight
                continue
            self.stats["decode_tokens"] += 1
            self._accept_token(r, int(t), now)
        t3 = time.perf_counter()
        self.stats["decode_host_s"] = self.stats.get("decode_host_s", 0.0) + (t3 - t2)
        self.stats["decode_gpu_wait_s"] = self.stats.get("decode_gpu_wait_s", 0.0) + (t2 - t1)

    # ------------------------------------------------------------------ decode
    def _reserve_decode(self) -> list:
        """Reserve one cache slot per running sequence and fill the host decode buffers (ids, positions,
        slots, context lengths, block tables) in one native call; when the pool is dry the youngest
        running sequence is preempted (recompute) and the call retried.  -> the decode batch."""
        while True:
            batch = list(self.running)
            B = len(batch)
            if B == 0:
                return batch
            fail = self.blocks.prepare_decode_into(
                [r.seq for r in batch], [r.out[-1] for r in batch], self.max_blocks_per_seq,
                self._h_ids.data_ptr(), self._h_pos.data_ptr(), self._h_slots.data_ptr(), self._h_ctx.data_ptr(),
                self._h_bt.data_ptr())
            if fail < 0:
                return batch
            if not self._preempt_one(protect=None if B == 1 else batch[fail]):
                raise RuntimeError("KV cache exhausted")

    def _run_decode(self, batch: list):
        t0 = time.perf_counter()
        B = len(batch)
        self._h_temp[:B] = torch.tensor([r.params.temperature if r.params.do_sample else 0.0 for r in batch])
        self._h_topk[:B] = torch.tensor([r.params.top_k for r in batch], dtype=torch.int32)
        self._h_topp[:B] = torch.tensor([r.params.top_p for r in batch])
        self._h_cnt[:B] = torch.tensor([r.rng_base + len(r.out) for r in batch], dtype=torch.int64)
        self._fast = all((0 < r.params.top_k <= ops.kernels.SAMPLE_FAST_MAX_K) or not r.params.do_sample
                         or r.params.temperature <= 0 for r in batch)
        Bp = next(b for b in self._buckets if b >= B) if self.use_graphs else B
        if Bp > B:  # padding rows: no cache write, attend to one key of block 0, output ignored
            self._h_ids[B:Bp] = 0
            self._h_pos[B:Bp] = 0
            self._h_slots[B:Bp] = -1
            self._h_ctx[B:Bp] = 1
            self._h_bt[B:Bp] = 0
            self._h_temp[B:Bp] = 0.0
            self._h_topk[B:Bp] = 1
            self._h_topp[B:Bp] = 1.0
            self._h_cnt[B:Bp] = 0
        self._fill_order(Bp)
        for d, h in ((self._d_ids, self._h_ids), (self._d_pos, self._h_pos), (self._d_slots, self._h_slots),
                     (self._d_ctx, self._h_ctx), (self._d_temp, self._h_temp), (self._d_topk, self._h_topk),
                     (self._d_topp, self._h_topp), (self._d_cnt, self._h_cnt), (self._d_order, self._h_order)):
            d[:Bp].copy_(h[:Bp], non_blocking=True)
        self._d_bt[:Bp].copy_(self._h_bt[:Bp], non_blocking=True)
        self._masked = self._fill_masks(batch, Bp)
        t1 = time.perf_counter()
        g = None
        # (vocab-parallel full-vocabulary sampling gathers the logits in the body: eager)
        if self.use_graphs and not (self.vp and not self._fast):
            g = self._graphs.get((Bp, self._fast, self._masked))
            if g is None:
                g = self._capture(Bp)
        with self.timer.phase("decode"):
            if g is not None:
                g.replay()
                self.stats["graph_replays"] += 1
            else:
                self._decode_body(Bp)
        if self.is_gpu:
            if self.vp and self._fast:
                self._vp_merge(self._vp_cand[:, :Bp], self._d_temp[:Bp], self._d_topk[:Bp], self._d_topp[:Bp],
                               self._d_cnt[:Bp], out=self._d_tokens[:Bp])
            else:
                self._tp_sync_tokens(self._d_tokens[:Bp])
            self._h_tokens[:Bp].copy_(self._d_tokens[:Bp], non_blocking=True)
            self._tp_fault_enqueue()
            torch.cuda.current_stream(self.device).synchronize()
            self._tp_fault_check()  # before any token of this step is accepted
        t2 = time.perf_counter()
        self._collect_gpu_times()
        toks = self._h_tokens[:B].tolist()
        now = time.perf_counter()
        self.stats["decode_steps"] += 1
        self.stats["decode_tokens"] += B
        for r, t in zip(batch, toks):
            self._accept_token(r, int(t), now)
        t3 = time.perf_counter()
        self.stats["decode_host_s"] = self.stats.get("decode_host_s", 0.0) + (t1 - t0) + (t3 - t2)
        self.stats["decode_gpu_wait_s"] = self.stats.get("decode_gpu_wait_s", 0.0) + (t2 - t1)

    def _fill_order(self, Bp: int) -> None:
        """Host: the decode attention's dispatch order for this step, longest context first (LPT
        balance of the two workgroup rounds per CU; benchmarks/decode_attn_bench.py)."""
        ctx = self._h_ctx[:Bp].numpy()
        self._h_order[:Bp] = torch.from_numpy(np.argsort(-ctx, kind="stable").astype(np.int32))

    def _decode_part(self, Bp: int) -> int:
        """Decode attention key partition for a step of Bp sequences: long partitions once the
        (sequence, kv head) pairs alone cover every CU twice over (512 pairs on 256 CUs).  (At batch
        1 the attention is a chain of dependent round trips: 16.4 us per layer with 512- and with
        128-key partitions alike, profiles/low_load_latency.md.)"""
        hkv = self.cfg.kv_heads // self.tp_size
        return self.long_part_size if Bp * hkv >= 512 else self.part_size

    def _decode_body(self, Bp: int):
        meta = AttnMeta(decode=True, positions=self._d_pos[:Bp], slots=self._d_slots[:Bp],
                        block_tables=self._d_bt[:Bp], ctx_lens=self._d_ctx[:Bp], workspace=self._workspace,
                        part_size=self._decode_part(Bp), order=self._d_order[:Bp] if self.is_gpu else None)
        h = self.model.forward(self._d_ids[:Bp], meta, self.kv)
        logits = self.model.logits(h)
        if self._masked:
            self._mask(logits, Bp)
        if self.is_gpu and self.vp and self._fast:
            # this rank's candidates; the all-gather + merge follow the replay (_run_decode)
            ops.sample_candidates(logits, self.model.vocab_local, self.model.vocab_start, out=self._vp_cand[:, :Bp])
        elif self.is_gpu:
            if self.vp:
                logits = self.model.full_logits(logits)
            ops.sample_tokens(logits, self._d_temp[:Bp], self._d_topk[:Bp], self._d_topp[:Bp], self.seed,
                              self._d_cnt[:Bp], out=self._d_tokens[:Bp], fast=self._fast,
                              workspace=self._sample_ws)
        else:
            if self.vp:
                logits = self.model.full_logits(logits)
            g = torch.Generator().manual_seed(int(self.seed * 7919 + int(self._h_cnt[0])))
            self._d_tokens[:Bp] = ops.sample_tokens(logits, self._d_temp[:Bp], self._d_topk[:Bp], self._d_topp[:Bp],
                                                    self.seed, self._d_cnt[:Bp], generator=g)
            self._h_tokens[:Bp] = self._d_tokens[:Bp]

    def _capture(self, Bp: int):
        try:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                self._decode_body(Bp)  # warm-up (allocator, lazy init) outside the graph
            torch.cuda.current_stream(self.device).wait_stream(s)
            torch.cuda.synchronize(self.device)
            self._d_cnt[:Bp].copy_(self._h_cnt[:Bp])  # the warm-up advanced the RNG counters
            g = torch.cuda.CUDAGraph()
            if self._graph_pool is None:
                self._graph_pool = torch.cuda.graph_pool_handle()
            with torch.cuda.graph(g, pool=self._graph_pool, stream=s):
                self._decode_body(Bp)
            torch.cuda.synchronize(self.device)
            self._graphs[(Bp, self._fast, self._masked)] = g
            return g
        except Exception as exc:  # pragma: no cover - depends on the runtime
            import logging

            logging.getLogger(__name__).warning("HIP graph capture failed (%s); decode runs eagerly", exc)
            self.use_graphs = False
            return None

    def capture_all(self, sizes=None):
        self._fast = True
        self._masked = False
        for b in sizes or self._buckets:
            if (b, True, False) not in self._graphs:
                self._capture(b)
