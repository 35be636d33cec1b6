#!/usr/bin/env python
"""Headline benchmark: RAG queries/sec + p50 end-to-end latency, bge-base + Llama-3-8B (BASELINE.json).

Every question goes through the engine's RAG path (``django_assistant_bot_amd.engine.rag.RAGPipeline``,
the batched mirror of the reference's ContextService -> ChatCompletion chain):

    bge-base query embedding (native encoder kernels)
    -> exact top-250 question search over a 1M-row in-HBM index (fused MFMA score GEMM + radix top-k)
    -> per-document aggregation (max_scores_n=5, top_n=5) -> FillInfo (<= 3 docs, 15 % of 8000)
    -> FinalPrompt -> Llama-3-8B generation of a fixed number of tokens (ignore_eos) with the
       reference's sampling (temperature 1, top_k 50, top_p 0.95), continuous batching + paged KV +
       HIP-graph decode.

Two load shapes (``--mode``):

  * ``batch`` (default) -- one step = a batch of C (= ``--batch``) questions answered together
    (retrieve all, prefill all, decode all); the index is sharded across the ranks (queries
    all-gathered, partial top-k routed back with all_to_all).  Driver record of round 3 at C=128 on
    one MI355X: 38.45 q/s, p50 3.33 s (BENCH_r03.json).
  * ``serve`` -- a bot's real traffic: questions keep arriving.  Closed loop at a fixed
    concurrency C per replica (whenever ``--admit-group`` slots are free, that many new questions
    are retrieved and queued), or open loop at ``--qps`` arrivals per second per replica (latency
    from the scheduled arrival, queueing included).  Admitted prompts are prefilled in their own
    steps by default (``--mixed-tokens 0``; mixing prompt chunks into decode steps measured slower,
    profiles/serving_mixed_steps.md).  One "step" = C completed questions.  The index is replicated
    per GPU (1.5 GB of 288 GB), so retrieval never waits on another rank.
  * ``overlap`` -- two engines sharing one weight copy on two streams (throughput setting).

Configs (``--config``, BASELINE.json): 4 (default) is the headline above; 5 is bge-large +
Llama-3-70B with TP = --gpus in serve mode at a fixed QPS.

Weights are random-init with the real architectures; corpus / questions are synthetic: each
question has planted "paraphrase" rows near its embedding in 3-5 target documents so retrieval
returns real documents and prompts have realistic length (~1k tokens).  Every rank runs TP=1 by
default (DP replicas; "scaling": weak -- per-GPU load fixed).

    python bench.py --gpus N --steps K --warmup W

With N > 1 and no torch.distributed.run around it, bench.py starts the N ranks itself
(``parallel/launch.py``: torch.distributed.run as a child process, rendezvous on 127.0.0.1) and
forwards rank 0's JSON line; under torch.distributed.run it is one rank.  ``n_gpus`` is the world
that formed; a mismatch with --gpus is an error.  ``DAB_DIST_BACKEND=gloo`` rehearses N ranks on one
GPU (RCCL needs one device per rank).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "RAG queries/sec + p50 end-to-end latency, bge-base + Llama-3-8B, 1/2/4/8 MI355X"
# No published reference number; BASELINE.md's comparison point is the measured re-run of the
# reference algorithm (benchmarks/reference_rerun.py, profiles/reference_rerun.md): 0.277 q/s per
# gunicorn worker on one MI355X, x2 for its default of 2 workers (upper bound) -> per GPU.
BASELINE_QPS_PER_GPU = 0.554
METRIC_CONFIG5 = "RAG queries/sec + p50 end-to-end latency at fixed QPS, bge-large + Llama-3-70B TP=8 (config 5)"

_WORDS = ("account access admin answer api archive backup billing bot calendar campaign channel client cloud "
          "config contact contract dashboard data deadline delivery deploy dialog document domain email error "
          "export feature file filter form group guide invoice issue key language limit list login message "
          "metric model module network notification order owner password payment plan policy price profile "
          "project query queue quota refund region report request role schedule search server service session "
          "setting storage subscription support task team template ticket token topic update upload user "
          "version webhook wiki workflow").split()


def synth_text(rng: np.random.Generator, n_words: int) -> str:
    w = rng.choice(len(_WORDS), n_words)
    out = []
    for i, j in enumerate(w):
        out.append(_WORDS[j])
        if i % 13 == 12:
            out[-1] += "."
    return " ".join(out)


class SyntheticDocuments(dict):
    """Document store: doc id -> StoredDocument with ~200-300 words.  ``materialize`` builds every
    document up front (an in-memory store, like the rows a deployment would fetch from its database);
    otherwise documents are generated on first access."""

    def __init__(self, n_docs: int, seed: int):
        super().__init__()
        self.n_docs, self.seed = n_docs, seed

    def materialize(self):
        """All documents at once: word ids for the whole corpus in one draw, then one join per
        document (every 13th word ends a sentence)."""
        from django_assistant_bot_amd.engine.rag import StoredDocument

        rng = np.random.default_rng(self.seed * 7919 + 17)
        lens = rng.integers(200, 300, self.n_docs)
        offs = np.concatenate([[0], np.cumsum(lens)])
        words = rng.integers(0, len(_WORDS), int(offs[-1]))
        pos = np.arange(int(offs[-1])) - np.repeat(offs[:-1], lens)
        vocab = np.array(list(_WORDS) + [w + "." for w in _WORDS], dtype=object)
        toks = vocab[words + len(_WORDS) * (pos % 13 == 12)].tolist()
        for k in range(self.n_docs):
            dict.__setitem__(self, k, StoredDocument(k, f"Document {k}", f"Wiki / Section {k // 100} / Document {k}",
                                                     " ".join(toks[offs[k]:offs[k + 1]])))
        return self

    def __contains__(self, k):
        return 0 <= int(k) < self.n_docs

    def __getitem__(self, k):
        from django_assistant_bot_amd.engine.rag import StoredDocument

        k = int(k)
        if not dict.__contains__(self, k):
            rng = np.random.default_rng(self.seed * 7919 + k)
            dict.__setitem__(self, k, StoredDocument(k, f"Document {k}", f"Wiki / Section {k // 100} / Document {k}",
                                                     synth_text(rng, int(rng.integers(200, 300)))))
        return dict.__getitem__(self, k)


SYSTEM_TEXT = ("You are a helpful assistant of the company support team. Answer the user's questions about the "
               "product, their account, billing and settings politely and precisely, in the user's language. "
               "Use only the information provided to you, keep answers short and structured, and never invent "
               "facts, prices, dates or links. If the question is unclear, ask the user to clarify it.")


def measure_fast_steps(rag, llm, questions, info, dev, classify_tokens: int = 16, known_tokens: int = 8,
                       n_topics: int = 12):
    """The reference answers every RAG query after two fast-model JSON calls: ClassifyStep
    (/root/reference/assistant/bot/services/context_service/steps/classify.py:41-45, <= 256 tokens)
    and ChooseKnownQuestionStep (.../steps/choose_known_question.py:45-50).  Both run here with the
    same prompt builders as the app layer (assistant.bot.services.context_service.steps), batched
    over the questions of one batch on the same engine, back to back, in JSON mode (constrained
    decoding: one generation per answer where the reference retries up to 5 times).  With
    random-init weights the JSON answers have no natural length, so the budget is that of a
    schema-valid answer ({"topic": "<title>"} ~ 16 tokens, {"question": <n>} ~ 8 tokens); an answer
    ends when its object closes.  Returns seconds per batch (max over ranks), the prompt sizes and
    the fraction of answers that parse."""
    from assistant.bot.services.context_service.steps.choose_known_question import ChooseKnownQuestionStep
    from assistant.bot.services.context_service.steps.classify import ClassifyStep
    from assistant.bot.services.context_service.utils import add_system_message
    from django_assistant_bot_amd.engine.llm_engine import SamplingParams
    from django_assistant_bot_amd.engine.rag import render_messages
    from django_assistant_bot_amd.parallel import dist as pdist

    trng = np.random.default_rng(4242)
    topics = ["Small talk"] + [f"Section {i}" for i in range(n_topics)]
    examples = list(ClassifyStep._offtopic_examples) + [
        (synth_text(trng, 10) + "?", t) for t in topics[1:] for _ in range(2)]

    def row_question(row_id: int) -> str:  # the text of an index row (a generated question)
        return synth_text(np.random.default_rng(10_000_019 + int(row_id)), 10) + "?"

    def encode(prompts):
        flat, offs = llm.tokenizer.encode_batch(prompts, add_special=True, max_len=llm.max_model_len - 1)
        flat, offs = np.asarray(flat), np.asarray(offs)
        return [flat[offs[i]:offs[i + 1]].tolist() for i in range(len(prompts))]

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    pdist.barrier(info)
    sync()
    t0 = time.perf_counter()
    base = [[{"role": "system", "content": SYSTEM_TEXT}, {"role": "user", "content": q}] for q in questions]
    cls_prompts = encode([render_messages(add_system_message(m, ClassifyStep.prompt(topics, examples, q)))
                          for m, q in zip(base, questions)])
    outs = llm.generate(cls_prompts, SamplingParams(max_new_tokens=classify_tokens, ignore_eos=True, json_mode=True))
    sync()
    t1 = time.perf_counter()
    related = [[int(x.split()[0][1:]) for x in dbg["related_questions"]] for _, dbg in rag.retrieve(questions, 0)]
    kq_prompts = encode([render_messages(add_system_message([], ChooseKnownQuestionStep.prompt(
        q, [row_question(r) for r in rel[:5]]))) for q, rel in zip(questions, related)])
    outs += llm.generate(kq_prompts, SamplingParams(max_new_tokens=known_tokens, ignore_eos=True, json_mode=True))
    sync()
    t2 = time.perf_counter()

    def parses(text):
        try:
            return isinstance(json.loads(text), dict)
        except ValueError:
            return False
    cls_s = pdist.max_over_ranks(t1 - t0, dev)
    kq_s = pdist.max_over_ranks(t2 - t1, dev)
    return {"classify_s": round(cls_s, 4), "known_question_s": round(kq_s, 4), "total_s": round(cls_s + kq_s, 4),
            "classify_prompt_tokens": int(np.mean([len(p) for p in cls_prompts])),
            "known_question_prompt_tokens": int(np.mean([len(p) for p in kq_prompts])),
            "answer_tokens": [classify_tokens, known_tokens], "batch": len(questions),
            "json_valid": round(float(np.mean([parses(o.text) for o in outs])), 4),
            "json_mean_tokens": round(float(np.mean([len(o.token_ids) for o in outs])), 2)}


def _host_profiler():
    """cProfile of the first timed batch's host side when DAB_HOST_PROFILE names an output file
    (finds the host work that leaves the GPU idle between the query embedding and the prefill)."""
    if not os.environ.get("DAB_HOST_PROFILE"):
        return None
    import cProfile

    prof = cProfile.Profile()
    prof.enable()
    return prof


def _dump_host_profile(prof):
    import io
    import pstats

    prof.disable()
    buf = io.StringIO()
    st = pstats.Stats(prof, stream=buf).sort_stats("cumulative")
    st.print_stats(60)
    st.sort_stats("tottime").print_stats(40)
    with open(os.environ["DAB_HOST_PROFILE"], "w") as f:
        f.write(buf.getvalue())


class _Heartbeat:
    """Rank 0 writes '[bench] <phase> <elapsed>' to stderr when a phase starts and every 60 s
    after, so a long setup (a 70B TP rehearsal builds 8 ranks' shards on one card) is visibly alive;
    stdout keeps only the one JSON line."""

    def __init__(self, rank: int):
        import threading

        self.rank, self.t0, self.name = rank, time.perf_counter(), ""
        if rank == 0:
            threading.Thread(target=self._beat, daemon=True).start()

    def __call__(self, name: str) -> None:
        self.name = name
        if self.rank == 0:
            print(f"[bench] {name} ({time.perf_counter() - self.t0:.0f} s)", file=sys.stderr, flush=True)

    def _beat(self):
        while True:
            time.sleep(60)
            print(f"[bench] ... {self.name} ({time.perf_counter() - self.t0:.0f} s)", file=sys.stderr, flush=True)


def _apply_config(args, ap) -> None:
    """BASELINE.json config presets.  Config 5 (Llama-3-70B TP=8 + bge-large at a fixed QPS) takes
    its TP degree from --gpus; flags given explicitly on the command line keep their value (a
    rehearsal swaps in a tiny-depth 70B layout with --llm-model)."""
    if args.config != 5:
        return
    given = {a.split("=")[0] for a in sys.argv[1:] if a.startswith("--")}
    preset = {"llm_model": "llama-3-70b", "embed_model": "bge-large-en", "mode": "serve", "qps": 4.0,
              "batch": 64, "tp": args.gpus}
    for k, v in preset.items():
        if "--" + k.replace("_", "-") not in given:
            setattr(args, k, v)
    if args.mode != "serve" or args.qps <= 0:
        ap.error("--config 5 is an open-loop serve run: --mode serve with --qps > 0")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--mode", choices=("serve", "batch", "overlap"), default="batch",
                    help="overlap: two engines sharing the weights on two streams, batches alternating "
                         "so one's prefill overlaps the other's decode (throughput setting)")
    ap.add_argument("--batch", type=int, default=128,
                    help="questions in flight per GPU (serve) / per batch (batch); one step = this many answers")
    ap.add_argument("--admit-group", type=int, default=32, help="serve: questions retrieved + queued together")
    ap.add_argument("--qps", type=float, default=0.0,
                    help="serve: open-loop arrivals at this rate per replica (fixed-QPS load, BASELINE config 5); "
                         "latency then counts from the scheduled arrival, queueing included")
    ap.add_argument("--mixed-tokens", type=int, default=0,
                    help="serve: prompt tokens mixed into one decode step (0, the default: separate prefill "
                         "steps; 2048 mixed measured 35.7 vs 38.4 q/s, profiles/serving_mixed_steps.md)")
    ap.add_argument("--max-new-tokens", type=int, default=256)
    ap.add_argument("--prefill-tokens", type=int, default=32768, help="prompt tokens per prefill step")
    ap.add_argument("--index-rows", type=int, default=1_000_000, help="question rows in the whole (sharded) index")
    ap.add_argument("--rows-per-doc", type=int, default=10)
    ap.add_argument("--embed-model", default="bge-base-en")
    ap.add_argument("--llm-model", default="llama-3-8b")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--kv-gb", type=float, default=None)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel size (groups of consecutive ranks)")
    ap.add_argument("--no-fast-steps", action="store_true",
                    help="skip the separately reported classify / known-question generations")
    ap.add_argument("--config", type=int, choices=(4, 5), default=4,
                    help="BASELINE config: 4 = bge-base + Llama-3-8B, TP=1 per GPU, batch mode (the headline); "
                         "5 = bge-large + Llama-3-70B, TP = --gpus, serve mode at a fixed QPS (--qps, default 4)")
    args = ap.parse_args()
    _apply_config(args, ap)

    # --gpus N from a plain process: start the N ranks here (children of this process, which has
    # not touched the GPU) and exit with the job's code; under torch.distributed.run this is a rank
    from django_assistant_bot_amd.parallel.launch import check_world, maybe_spawn

    maybe_spawn(args.gpus, __file__)

    from django_assistant_bot_amd.engine.embedding_engine import EmbeddingEngine
    from django_assistant_bot_amd.engine.llm_engine import LLMEngine, SamplingParams
    from django_assistant_bot_amd.engine.rag import RAGPipeline
    from django_assistant_bot_amd.engine.vector_index import VectorIndex
    from django_assistant_bot_amd.parallel import dist as pdist
    from django_assistant_bot_amd.parallel.sharded_index import ShardedIndex

    info = pdist.init()
    dev = info.device
    W, R = info.world_size, info.rank
    tp_group, tp_rank, rep = pdist.tp_groups(args.tp)
    if args.tp > 1:
        rep = R // args.tp  # DP replica index (consecutive ranks form a TP group)
    n_rep = W // max(1, args.tp)
    check_world(args.gpus, W)
    if W % max(1, args.tp):
        raise SystemExit(f"--tp {args.tp} does not divide the world of {W} ranks")
    torch.manual_seed(args.seed + R)
    B = args.batch
    n_steps = args.warmup + args.steps

    serve = args.mode == "serve"
    overlap = args.mode == "overlap"
    if overlap and (args.warmup < 2 or args.tp > 1):
        raise SystemExit("--mode overlap needs --warmup >= 2 (one batch per engine) and --tp 1")
    G = max(1, min(args.admit_group, B))
    if serve:
        # questions answered in the timed window + the ones still in flight at both ends
        n_questions = n_steps * B + 2 * B
    else:
        n_questions = n_steps * B

    t_setup = time.perf_counter()
    phase = _Heartbeat(R)
    phase("setup: engines")
    embedder = EmbeddingEngine(args.embed_model, dev, seed=args.seed)
    kv_gb = args.kv_gb if (args.kv_gb or not overlap) else 48.0  # two pools in overlap mode
    llm = LLMEngine(args.llm_model, dev, seed=args.seed + 17 * rep, max_batch=B, max_model_len=4096,
                    use_graphs=not args.no_graphs, kv_cache_gb=kv_gb, max_prefill_tokens=args.prefill_tokens,
                    mixed_prefill_tokens=args.mixed_tokens if serve else 0, tp_group=tp_group, tp_size=args.tp,
                    tp_rank=tp_rank)
    llm2 = None
    if overlap:
        llm2 = LLMEngine(args.llm_model, dev, seed=args.seed + 17 * rep, max_batch=B, max_model_len=4096,
                         use_graphs=not args.no_graphs, kv_cache_gb=kv_gb, max_prefill_tokens=args.prefill_tokens,
                         shared_model=llm.model)
    phase("setup: index")
    # ---- synthetic corpus: index rows (questions) grouped into documents
    n_rows = args.index_rows
    n_docs = max(1, n_rows // args.rows_per_doc)
    docs = SyntheticDocuments(n_docs, args.seed).materialize()
    if serve or overlap:  # replicated: every rank holds all rows (identical generator), no collective per search
        index = VectorIndex(embedder.dim, dev)
        gen = torch.Generator(device=dev).manual_seed(args.seed * 31)
        my_ids = np.arange(n_rows, dtype=np.int64)
    else:
        index = ShardedIndex(embedder.dim, dev)
        gen = torch.Generator(device=dev).manual_seed(args.seed * 31 + R)
        my_ids = np.arange(R, n_rows, W, dtype=np.int64)
    chunk = 1 << 18
    for s in range(0, len(my_ids), chunk):
        ids = my_ids[s:s + chunk]
        v = torch.randn((len(ids), embedder.dim), device=dev, generator=gen)
        index.add(ids, v, doc_ids=ids // args.rows_per_doc, groups=np.zeros(len(ids), dtype=np.int32))
    # ---- questions of every replica (deterministic), embedded once to plant relevant rows
    qrng = np.random.default_rng(args.seed + 12345)
    all_q = [[synth_text(qrng, int(qrng.integers(8, 16))) + "?" for _ in range(n_questions)] for _ in range(n_rep)]
    flat_q = [q for r in all_q for q in r]
    q_emb = torch.cat([embedder.embed(flat_q[i:i + 4096]).float() for i in range(0, len(flat_q), 4096)])
    q_emb = torch.nn.functional.normalize(q_emb, dim=-1)
    # Random-init encoders embed every question into a narrow cone (pairwise cos ~0.96), so rows
    # planted at q + noise would also match the OTHER questions and the hit lists would depend on how
    # many questions were planted (i.e. on --batch).  Planting along each question's own component
    # off the common direction (q + beta * (q - (q.mu) mu)) keeps its rows ~0.13 closer to it than to
    # any other question: every query then retrieves its own 3-5 documents at any batch size.
    mu = torch.nn.functional.normalize(q_emb.mean(0), dim=0)
    q_own = q_emb - (q_emb @ mu)[:, None] * mu[None]
    beta = 3.0
    prng = np.random.default_rng(args.seed + 999)
    plant_ids, plant_vecs, plant_docs = [], [], []
    for qi in range(len(flat_q)):
        n_t = int(prng.integers(3, 6))
        targets = prng.choice(n_docs, n_t, replace=False)
        for rank_t, d in enumerate(targets):
            rows = d * args.rows_per_doc + np.arange(min(args.rows_per_doc, 6))
            rows = rows[rows < n_rows]
            sigma = 0.02 + 0.004 * rank_t  # distance ~0.18: broad-search path, not the 0.05 shortcut
            noise = torch.randn((len(rows), embedder.dim), device=dev, generator=torch.Generator(device=dev)
                                .manual_seed(qi * 10 + rank_t)) * sigma
            plant_ids.append(rows)
            plant_vecs.append((q_emb[qi] + beta * q_own[qi])[None] + noise)
            plant_docs.append(np.full(len(rows), d, dtype=np.int64))
    index.add(np.concatenate(plant_ids), torch.cat(plant_vecs), doc_ids=np.concatenate(plant_docs),
              groups=np.zeros(sum(len(x) for x in plant_ids), dtype=np.int32))
    del q_emb, q_own
    rag_lock = threading.Lock() if overlap else None
    rag = RAGPipeline(embedder, index, llm, docs, system_text=SYSTEM_TEXT, retrieve_lock=rag_lock)
    rag2 = RAGPipeline(embedder, index, llm2, docs, system_text=SYSTEM_TEXT, retrieve_lock=rag_lock) if overlap else None
    if overlap and llm.use_graphs:  # no capture may run while the other engine's thread launches work
        llm.capture_all()
        llm2.capture_all()
    params = SamplingParams(max_new_tokens=args.max_new_tokens, ignore_eos=True, temperature=1.0, top_k=50,
                            top_p=0.95)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    setup_s = time.perf_counter() - t_setup
    phase("warm-up and timed steps")

    def sync_start():
        pdist.barrier(info)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        return dict(llm.stats), time.perf_counter()

    latencies, prompt_lens, n_docs_used = [], [], []
    phases = {"retrieve_s": [], "prompt_s": [], "generate_s": []}
    my_q = all_q[rep]
    if serve:
        # closed loop at concurrency B; during the ramp one group is admitted every
        # max_new_tokens * G / B decode steps so completions are spread evenly from then on
        pace = max(1, args.max_new_tokens * G // B)
        next_q, next_admit, admitted, done = 0, 0, 0, 0
        warm_n, total_n = args.warmup * B, n_steps * B
        t0 = None
        stats0, t0 = (sync_start() if warm_n == 0 else (None, None))
        arrival_of: dict = {}
        t_open = time.perf_counter()
        while done < total_n:
            if args.qps > 0:  # open loop: everything scheduled to have arrived by now is submitted
                due = min(len(my_q), int((time.perf_counter() - t_open) * args.qps) + 1)
                if args.tp > 1:  # the TP group's engines must admit the same requests at the same step
                    due = pdist.broadcast_int(due, tp_group, dev)
                if due > next_q:
                    rids = rag.submit(my_q[next_q:due], params, bot_group=0)
                    for j, rid in enumerate(rids):
                        arrival_of[rid] = t_open + (next_q + j) / args.qps
                    admitted += due - next_q
                    next_q = due
            while (args.qps <= 0 and rag.in_flight + G <= B and next_q + G <= len(my_q)
                   and (admitted >= B or llm.stats["decode_steps"] >= next_admit)):
                rag.submit(my_q[next_q:next_q + G], params, bot_group=0)
                next_q += G
                admitted += G
                next_admit += pace
            for rid, r in rag.poll():
                done += 1
                if t0 is not None:
                    sched = arrival_of.pop(rid, None)
                    latencies.append(time.perf_counter() - sched if sched is not None else r.latency_s)
                    prompt_lens.append(r.usage["prompt_tokens"])
                    n_docs_used.append(len(r.documents))
                    phases["retrieve_s"].append(r.debug_info["took"])
                    phases["prompt_s"].append(r.debug_info["prompt"]["took"])
                    phases["generate_s"].append(r.debug_info["final"]["took"])
                if done == warm_n and t0 is None:
                    stats0, t0 = sync_start()
                if done == total_n:
                    break
    elif overlap:
        # warm-up batches alternate between the engines on the main thread; then one thread per
        # engine, each on its own stream, works through its half of the timed batches; engine 1
        # starts once engine 0's first timed batch is decoding, so their phases interleave
        pipes = (rag, rag2)
        for step in range(args.warmup):
            pipes[step % 2].answer(my_q[step * B:(step + 1) * B], params, bot_group=0)
        stats0, t0 = sync_start()
        go = threading.Event()
        results = ([], [])
        errors = []

        def run(w):
            import contextlib

            try:
                gpu = dev.type == "cuda"
                if gpu:
                    torch.cuda.set_device(dev)
                pipe = pipes[w]
                if w == 1:
                    go.wait(timeout=600)
                with torch.cuda.stream(torch.cuda.Stream(dev)) if gpu else contextlib.nullcontext():
                    for step in range(args.warmup + w, n_steps, 2):
                        qs = my_q[step * B:(step + 1) * B]
                        rids = pipe.submit(qs, params, bot_group=0)
                        pending, got = set(rids), {}
                        while pending:
                            for rid, r in pipe.poll():
                                got[rid] = r
                                pending.discard(rid)
                            if w == 0 and not go.is_set() and pipe.llm.running and not (
                                    pipe.llm.waiting or pipe.llm.prefilling):
                                go.set()
                        results[w].append([got[r] for r in rids])
                        go.set()
                    if gpu:
                        torch.cuda.current_stream(dev).synchronize()
            except BaseException as exc:  # surfaced on the main thread
                errors.append(exc)
                go.set()

        threads = [threading.Thread(target=run, args=(w,)) for w in (0, 1)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errors:
            raise errors[0]
        for res in results[0] + results[1]:
            latencies += [r.latency_s for r in res]
            prompt_lens += [r.usage["prompt_tokens"] for r in res]
            n_docs_used += [len(r.documents) for r in res]
            phases["retrieve_s"].append(res[0].debug_info["took"])
            phases["prompt_s"].append(res[0].debug_info["prompt"]["took"])
            phases["generate_s"].append(max(r.debug_info["final"]["took"] for r in res))
    else:
        for step in range(n_steps):
            if step == args.warmup:
                stats0, t0 = sync_start()
            prof = _host_profiler() if step == args.warmup else None
            res = rag.answer(my_q[step * B:(step + 1) * B], params, bot_group=0)
            if prof is not None:
                _dump_host_profile(prof)
            if step >= args.warmup:
                latencies += [r.latency_s for r in res]
                prompt_lens += [r.usage["prompt_tokens"] for r in res]
                n_docs_used += [len(r.documents) for r in res]
                phases["retrieve_s"].append(res[0].debug_info["took"])
                phases["prompt_s"].append(res[0].debug_info["prompt"]["took"])
                phases["generate_s"].append(max(r.debug_info["final"]["took"] for r in res))
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    pdist.barrier(info)
    my_elapsed = time.perf_counter() - t0
    elapsed = pdist.max_over_ranks(my_elapsed, dev)
    rank_qps = [round(x, 3) for x in pdist.gather_floats(B * args.steps / my_elapsed, dev)]
    # engine counters of the timed region only (before the separately reported fast steps run)
    eng = {k: round(v - stats0.get(k, 0), 3) if isinstance(v, float) else v - stats0.get(k, 0)
           for k, v in llm.stats.items()}
    # ---- reported separately: the two fast JSON generations per query, after the
    # timed region so the headline is unchanged
    fast = None
    if not args.no_fast_steps and not serve and not overlap:
        fast = measure_fast_steps(rag, llm, my_q[:B], info, dev)
    p50 = float(np.median(latencies)) if latencies else float("nan")
    p50 = pdist.max_over_ranks(p50, dev)
    p90 = pdist.max_over_ranks(float(np.percentile(latencies, 90)) if latencies else float("nan"), dev)
    total_q = n_rep * B * args.steps
    qps = total_q / elapsed
    full = {}
    if fast:
        batch_s = elapsed / args.steps
        full = {"fast_steps_s": fast["total_s"],
                "full_pipeline_qps": round(n_rep * B / (batch_s + fast["total_s"]), 3),
                "full_pipeline_p50_latency_ms": round(1000 * (p50 + fast["total_s"]), 1)}
    cfg5 = args.config == 5
    tp_info = {}
    if args.tp > 1:
        hbm = [round(x / 2 ** 30, 2) for x in pdist.gather_floats(
            float(torch.cuda.max_memory_allocated(dev)) if dev.type == "cuda" else 0.0, dev)]
        tp_info = {"tp_allreduce_calls_rank0": dict(llm.model.ar_counts),
                   "tp_allreduce_note": "Python-issued calls; a call captured in a decode graph counts once",
                   "kv_blocks_rank0": int(llm.blocks.num_blocks()),
                   "hbm_peak_gb_per_rank": hbm}
    out = {
        "metric": METRIC_CONFIG5 if cfg5 else METRIC,
        "value": round(qps, 3),
        "unit": "queries/s",
        "n_gpus": W,
        "backend": info.backend,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * elapsed / args.steps, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None if cfg5 else round(qps / (BASELINE_QPS_PER_GPU * W), 2),
        "dtype": "bf16",
        "data": "synthetic (random-init weights; synthetic corpus/questions)",
        "p50_latency_ms": round(1000 * p50, 1),
        "p90_latency_ms": round(1000 * p90, 1),
        **full,
        "config": {
            "model": f"{args.embed_model} + {args.llm_model}",
            "global_batch": n_rep * B,
            "seq_len": int(np.mean(prompt_lens)) if prompt_lens else 0,
            "max_new_tokens": args.max_new_tokens,
            "parallelism": f"dp{n_rep}" + (f"xtp{args.tp}" if args.tp > 1 else ""),
            "mode": ("overlap (2 engines x batch {}, one weight copy, phases interleaved)".format(B) if overlap else
                     "batch" if not serve else
                     f"serve (open loop, {args.qps} q/s per replica offered, max batch {B}, mixed {args.mixed_tokens})"
                     if args.qps > 0 else
                     f"serve (closed loop, {B} in flight per replica, admit {G}, mixed {args.mixed_tokens})"),
            "index_rows": n_rows,
            # what ran: without a process group (world 1, no DAB_FORCE_GROUP) ShardedIndex.search
            # takes its local path and no collective is issued
            "index": ("replicated per GPU" if (serve or overlap) else
                      "sharded (all_to_all merge)" if index.distributed else "single shard, local top-k (no collective)"),
            "docs_per_prompt": round(float(np.mean(n_docs_used)), 2) if n_docs_used else 0,
            "sampling": "temperature=1.0 top_k=50 top_p=0.95 ignore_eos",
            "graphs": llm.use_graphs,
            "setup_s": round(setup_s, 1),
            "generated_tokens_per_s": round(total_q * args.max_new_tokens / elapsed, 1),
            "per_rank_qps": rank_qps,
            "engine_rank0": eng,
            **({"fast_steps": fast} if fast else {}),
            "phases_rank0_s": {k: round(float(np.mean(v)), 4) for k, v in phases.items() if v},
            **tp_info,
        },
    }
    if R == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    pdist.shutdown()


if __name__ == "__main__":
    main()
