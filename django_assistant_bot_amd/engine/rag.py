"""Batched RAG query path on the engine (embed -> search -> aggregate -> fill -> prompt -> generate).

This is the GPU-resident counterpart of the reference's per-message pipeline
(bot/services/context_service/service.py:43-52 and steps/*):

  EmbeddingsStep (steps/embeddings.py:19-66)
      query embedding; top-5 related questions; if the best question is closer than 0.05 the answer
      document is that question's document, otherwise the broad search: top
      ``max_scores_n * top_n * 10`` question hits aggregated per document (search_service.py:111-152,
      native ``aggregate_documents``).  The reference embeds the query twice (steps/embeddings.py:24 and
      search_service.py:127); here it is embedded once and ONE top-250 kernel call serves both searches
      (the related-question top-5 is the head of the same sorted list).
  FillInfoStep (steps/fill_info.py:10-33)
      at most 3 documents within 15 % of the generator context (8000 "tokens" = words // 2 estimate,
      ai/providers/gpu_service.py:16-20).
  FinalPromptStep (steps/final_prompt.py:13-45)
      system message with the documents, the current date and the answering rules.
  ChatCompletion (bot/chat_completion.py:24-45)
      the strong-model generation, here a batched call into ``LLMEngine``; prompt rendered as the
      reference's TransformersProvider does: ``"role: content"`` lines (ai/providers/transformers.py:50).

Everything for a whole batch of user questions happens in a handful of kernel launches.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from datetime import datetime

import numpy as np

from ..ops._lib import native
from ..utils import trace
from .llm_engine import LLMEngine, SamplingParams


@dataclass
class StoredDocument:
    id: int
    name: str
    path: str
    content: str


@dataclass
class RAGResult:
    question: str
    answer: str
    documents: list
    usage: dict
    finish_reason: str
    latency_s: float
    debug_info: dict = field(default_factory=dict)


def estimate_tokens(text: str) -> int:
    """The reference's crude token count for remote generators (ai/providers/gpu_service.py:19-20)."""
    return len(text.split()) // 2


def render_messages(messages: list[dict]) -> str:
    return "\n".join(f"{m['role']}: {m['content']}" for m in messages)


def final_info_message(final_info: str | None, question: str, now: datetime | None = None) -> str:
    if final_info is None:
        return ("Unfortunately, there is not enough information to answer the user's question for you.\n"
                "Answer the user that you could not help with the question.\n")
    now = now or datetime.now()
    return (
        "You must answer the user only using the following information:\n"
        f"```\n{final_info}\n# Current date: `{now.strftime('%Y-%m-%d %H:%M:%S')}`\n\n```\n"
        "As you remember, the question from the user is:\n"
        f"```\n{question}\n```\n"
        "If that information does not contain the answer, you must say that you don't have information like "
        "\"I'm sorry, I don't have enough information to answer your question.\" (but in user's language).\n"
        "Follow the original wording as much as possible.\n"
        "It would be ideal if your answer was an exact and complete quote from the document. "
        "Don't leave out details in your answer.\n"
    )


def fill_info(docs: list[StoredDocument], context_size: int = 8000, max_tokens_share: float = 0.15,
              max_documents: int = 3, count=estimate_tokens):
    """FillInfoStep semantics: returns (final_info or None, used documents)."""
    if not docs:
        return None, []
    budget = int(context_size * max_tokens_share)
    out, used = "", []
    for d in docs:
        if len(used) >= max_documents:
            break
        cand = f"{out}# {d.path}:\n```\n{d.content}\n```\n"
        if out and count(cand) > budget:
            break
        out = cand
        used.append(d)
    return out, used


class RAGPipeline:
    def __init__(self, embedder, index, llm: LLMEngine, documents: dict, system_text: str = "",
                 context_size: int = 8000, max_scores_n: int = 5, top_n: int = 5, related_n: int = 5,
                 same_question_distance: float = 0.05, max_documents: int = 3, max_tokens_share: float = 0.15,
                 retrieve_lock=None):
        """``retrieve_lock``: held around retrieval + prompt building when several pipelines (each
        with its own LLMEngine) share one embedder / index from different threads."""
        self.embedder, self.index, self.llm = embedder, index, llm
        self._retrieve_lock = retrieve_lock
        self.documents = documents
        self.system_text = system_text
        self.context_size = context_size
        self.max_scores_n, self.top_n, self.related_n = max_scores_n, top_n, related_n
        self.same_question_distance = same_question_distance
        self.max_documents, self.max_tokens_share = max_documents, max_tokens_share
        self._native = native()
        self._inflight: dict = {}
        self.timer = trace.GpuTimer(device=getattr(llm, "device", None))

    def retrieve(self, questions: list[str], bot_group: int | None = None):
        """-> per question (documents list, debug dict); one embed + one search for the whole batch."""
        t0 = time.perf_counter()
        with self.timer.phase("embed"):
            emb = self.embedder.embed(questions)
        t1 = time.perf_counter()
        k = self.max_scores_n * self.top_n * 10
        groups = None if bot_group is None else [bot_group] * len(questions)
        with self.timer.phase("search"):
            sims, ids, docs = self.index.search(emb, k, q_groups=groups)
        dist = (1.0 - sims).float().cpu().numpy()
        ids_h = ids.cpu().numpy()
        docs_h = docs.cpu().numpy()
        gpu_ms = {f"{k_}_gpu_ms": round(v, 3) for k_, v in self.timer.collect().items()}
        t2 = time.perf_counter()
        out = []
        for qi in range(len(questions)):
            valid = ids_h[qi] >= 0
            d, di = dist[qi][valid], docs_h[qi][valid]
            dbg = {"related_questions": [f"[{int(x)} {1 - float(y):.4f}]" for x, y in
                                         zip(ids_h[qi][valid][: self.related_n], d[: self.related_n])]}
            if len(d) and d[0] < self.same_question_distance:
                picked = [(int(di[0]), 1.0 - float(d[0]))]
                dbg["the_same_question"] = int(ids_h[qi][0])
            else:
                picked = self._native.aggregate_documents(d.astype(np.float32), di.astype(np.int64),
                                                          self.max_scores_n, self.top_n)
            seen, docs_q = set(), []
            for doc_id, score in picked:
                if doc_id in seen or doc_id not in self.documents:
                    continue
                seen.add(doc_id)
                docs_q.append(self.documents[doc_id])
            dbg["documents"] = [f"[{doc.id} {s:.4f}] {doc.name}" for doc, (_, s) in zip(docs_q, picked)]
            dbg["took"] = (t2 - t0)
            dbg["embed_s"] = t1 - t0
            dbg.update(gpu_ms)
            out.append((docs_q, dbg))
        return out

    def build_prompts(self, questions: list[str], retrieved, now: datetime | None = None):
        prompts, used_docs = [], []
        for q, (docs_q, _) in zip(questions, retrieved):
            info, used = fill_info(docs_q, self.context_size, self.max_tokens_share, self.max_documents)
            messages = []
            if self.system_text:
                messages.append({"role": "system", "content": self.system_text})
            messages.append({"role": "user", "content": q})
            messages.append({"role": "system", "content": final_info_message(info, q, now)})
            prompts.append(render_messages(messages))
            used_docs.append(used)
        flat, offs = self.llm.tokenizer.encode_batch(prompts, add_special=True, max_len=self.llm.max_model_len - 1)
        flat, offs = np.asarray(flat), np.asarray(offs)
        token_lists = [flat[offs[i]:offs[i + 1]].tolist() for i in range(len(prompts))]
        return token_lists, used_docs

    # -------------------------------------------------------------- serving (continuous arrival)
    def submit(self, questions: list[str], params: SamplingParams | None = None, bot_group: int | None = None,
               now: datetime | None = None) -> list[int]:
        """Retrieve + build prompts for newly arrived questions and queue their generations; answers
        come back from ``poll`` while earlier questions are still decoding (the engine mixes their
        prompt chunks into the running decode steps)."""
        params = params or SamplingParams(max_new_tokens=1024)
        t0 = time.perf_counter()
        if self._retrieve_lock is not None:
            with self._retrieve_lock:
                retrieved = self.retrieve(questions, bot_group)
                t_ret = time.perf_counter()
                token_lists, used_docs = self.build_prompts(questions, retrieved, now)
        else:
            retrieved = self.retrieve(questions, bot_group)
            t_ret = time.perf_counter()
            token_lists, used_docs = self.build_prompts(questions, retrieved, now)
        t_prompt = time.perf_counter()
        rids = []
        for q, toks, ret, used in zip(questions, token_lists, retrieved, used_docs):
            rid = self.llm.add_request(toks, params)
            self._inflight[rid] = (q, ret, used, t0, t_ret, t_prompt)
            rids.append(rid)
        return rids

    def poll(self) -> list[tuple[int, RAGResult]]:
        """One engine step -> (request id, result) of every question it completed."""
        out = []
        for rid in self.llm.step():
            if rid not in self._inflight:
                continue
            done = time.perf_counter()
            q, (docs_q, dbg), used, t0, t_ret, t_prompt = self._inflight.pop(rid)
            o = self.llm.pop_output(rid)
            dbg = dict(dbg)
            dbg["final"] = {"took": done - t_prompt, **o.timings}
            dbg["prompt"] = {"took": t_prompt - t_ret}
            dbg["total"] = {"took": done - t0}
            out.append((rid, RAGResult(q, o.text, [d.id for d in used], o.usage, o.finish_reason, done - t0, dbg)))
        return out

    @property
    def in_flight(self) -> int:
        return len(self._inflight)

    def answer(self, questions: list[str], params: SamplingParams | None = None, bot_group: int | None = None,
               now: datetime | None = None) -> list[RAGResult]:
        """Batch mode: answer a batch of questions end to end (submit + poll until all are done)."""
        rids = self.submit(questions, params, bot_group, now)
        pending = set(rids)
        got = {}
        while pending:
            for rid, res in self.poll():
                got[rid] = res
                pending.discard(rid)
        return [got[r] for r in rids]
