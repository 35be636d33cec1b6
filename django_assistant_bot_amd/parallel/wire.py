"""Fixed-shape control messages of the node / TP control planes: int64 tensors, no pickles.

Every message is a batch of items.  An item is one HDR-word int64 header (kind, ids, counts, numbers;
floats travel as their float64 bit patterns) plus an int64 payload whose length the header implies.
A batch goes over a gloo group as two tensors: ``meta`` = [n_items, payload_len] and one ``body`` =
the [n_items, HDR] header table followed by the concatenated payloads.  So a step's adds / aborts or
a replica's finished outputs cost two small sends, and no side needs to unpickle a peer's bytes.

Kinds used on the request links and inside TP groups (``parallel/node.py``, ``parallel/tp_serving.py``):

  ADD    [ADD, model, rid, n_prompt, n_stop, <sampling params>]  payload: prompt ids, stop ids
  ABORT  [ABORT, model, rid, n_reason]                            payload: reason bytes
  OUT    [OUT, model, rid, n_prompt, n_tokens, n_reason, <timings>] payload: prompt, tokens, reason
  STEP   [STEP, model]                                            (TP groups: step this model now)
  FAIL   [FAIL, model]                                            (drop every unfinished request)
  STOP   [STOP]
"""
from __future__ import annotations

import struct

import numpy as np
import torch
import torch.distributed as dist

HDR = 16
ADD, ABORT, OUT, STEP, FAIL, STOP = 1, 2, 3, 4, 5, 6
_NONE = -(1 << 62)  # "None" in an optional integer / float slot


def f2i(x: float) -> int:
    return struct.unpack("<q", struct.pack("<d", float(x)))[0]


def i2f(i: int) -> float:
    return struct.unpack("<d", struct.pack("<q", int(i)))[0]


def opt_i(x) -> int:
    return _NONE if x is None else int(x)


def i_opt(i: int):
    return None if int(i) == _NONE else int(i)


def opt_f(x) -> int:
    return _NONE if x is None else f2i(x)


def f_opt(i: int):
    return None if int(i) == _NONE else i2f(i)


def text_words(s: str) -> np.ndarray:
    return np.frombuffer(s.encode("utf-8"), dtype=np.uint8).astype(np.int64)


def words_text(a) -> str:
    return bytes(np.asarray(a, dtype=np.int64).astype(np.uint8).tolist()).decode("utf-8")


def item(words, payload=None):
    """(header int64[HDR], payload int64[n]) from a list of <= HDR ints and an int sequence."""
    h = np.zeros(HDR, dtype=np.int64)
    h[: len(words)] = np.asarray(words, dtype=np.int64)
    p = np.zeros(0, dtype=np.int64) if payload is None else np.asarray(payload, dtype=np.int64).reshape(-1)
    return h, p


def pack(items) -> tuple[torch.Tensor, torch.Tensor]:
    n = len(items)
    pays = [p for _, p in items]
    plen = int(sum(len(p) for p in pays))
    meta = torch.tensor([n, plen], dtype=torch.int64)
    if n == 0:
        return meta, torch.zeros(0, dtype=torch.int64)
    table = np.stack([h for h, _ in items])
    body = np.concatenate([table.reshape(-1)] + pays) if plen else table.reshape(-1)
    return meta, torch.from_numpy(np.ascontiguousarray(body))


def unpack(meta: torch.Tensor, body: torch.Tensor) -> list:
    n, _ = int(meta[0]), int(meta[1])
    if n == 0:
        return []
    b = body.numpy()
    table = b[: n * HDR].reshape(n, HDR)
    out, o = [], n * HDR
    for h in table:
        ln = payload_len(h)
        out.append((h.copy(), b[o:o + ln].copy()))
        o += ln
    return out


def payload_len(h) -> int:
    k = int(h[0])
    if k == ADD:
        return int(h[3]) + int(h[4]) + int(h[15])
    if k == ABORT:
        return int(h[3])
    if k == OUT:
        return int(h[3]) + int(h[4]) + int(h[5])
    return 0


# ---------------------------------------------------------------------- transports
def send_batch(items, dst: int, group) -> int:
    """Blocking point-to-point send of a batch; returns the bytes sent."""
    meta, body = pack(items)
    dist.send(meta, dst=dst, group=group)
    if int(meta[0]):
        dist.send(body, dst=dst, group=group)
    return 16 + body.numel() * 8


def recv_batch(src: int, group, meta: torch.Tensor | None = None) -> list:
    """Blocking receive of a batch (``meta`` already received by an ``irecv``, or not)."""
    if meta is None:
        meta = torch.zeros(2, dtype=torch.int64)
        dist.recv(meta, src=src, group=group)
    n, plen = int(meta[0]), int(meta[1])
    if n == 0:
        return []
    body = torch.zeros(n * HDR + plen, dtype=torch.int64)
    dist.recv(body, src=src, group=group)
    return unpack(meta, body)


def bcast_batch(items, src: int, group) -> list:
    """Broadcast a batch from ``src`` (global rank) over ``group``; every rank returns the items."""
    if items is not None:
        meta, body = pack(items)
    else:
        meta, body = torch.zeros(2, dtype=torch.int64), None
    dist.broadcast(meta, src=src, group=group)
    n, plen = int(meta[0]), int(meta[1])
    if n == 0:
        return []
    if body is None:
        body = torch.zeros(n * HDR + plen, dtype=torch.int64)
    dist.broadcast(body, src=src, group=group)
    return unpack(meta, body) if items is None else list(items)


# ---------------------------------------------------------------------- requests / outputs
def add_item(model: int, rid: int, prompt, params):
    stop = [int(t) for t in (params.stop_token_ids or ())]
    schema = np.zeros(0, dtype=np.int64)
    if params.json_schema is not None:
        from ..engine.json_schema import schema_key

        schema = text_words(schema_key(params.json_schema))
    words = [ADD, model, rid, len(prompt), len(stop), int(params.max_new_tokens), f2i(params.temperature),
             int(params.top_k), f2i(params.top_p), int(bool(params.ignore_eos)), opt_i(params.max_length),
             opt_i(params.seed), int(bool(params.do_sample)), opt_f(params.timeout_s), int(bool(params.json_mode)),
             len(schema)]
    return item(words, np.concatenate([np.asarray(list(prompt) + stop, dtype=np.int64), schema]))


def read_add(h, p):
    from ..engine.llm_engine import SamplingParams

    n_prompt, n_stop = int(h[3]), int(h[4])
    n_schema = int(h[15])
    schema = words_text(p[n_prompt + n_stop:n_prompt + n_stop + n_schema]) if n_schema else None
    sp = SamplingParams(max_new_tokens=int(h[5]), temperature=i2f(h[6]), top_k=int(h[7]), top_p=i2f(h[8]),
                        ignore_eos=bool(h[9]), max_length=i_opt(h[10]), seed=i_opt(h[11]),
                        stop_token_ids=tuple(int(t) for t in p[n_prompt:n_prompt + n_stop]), do_sample=bool(h[12]),
                        timeout_s=f_opt(h[13]), json_mode=bool(h[14]), json_schema=schema)
    return int(h[1]), int(h[2]), [int(t) for t in p[:n_prompt]], sp


def abort_item(model: int, rid: int, reason: str):
    r = text_words(reason)
    return item([ABORT, model, rid, len(r)], r)


def read_abort(h, p):
    return int(h[1]), int(h[2]), words_text(p)


_TIMINGS = ("queue_s", "ttft_s", "total_s", "decode_s", "prefill_s")


def out_item(model: int, out):
    """A finished ``GenerationOutput`` (text is re-decoded by the receiver's tokenizer)."""
    r = text_words(out.finish_reason)
    words = [OUT, model, out.request_id, len(out.prompt_ids), len(out.token_ids), len(r)]
    words += [f2i(out.timings.get(k, 0.0)) for k in _TIMINGS]
    return item(words, list(out.prompt_ids) + list(out.token_ids) + r.tolist())


def read_out(h, p, tokenizer):
    from ..engine.llm_engine import GenerationOutput

    n_p, n_t = int(h[3]), int(h[4])
    prompt = [int(t) for t in p[:n_p]]
    toks = [int(t) for t in p[n_p:n_p + n_t]]
    reason = words_text(p[n_p + n_t:])
    timings = {k: i2f(h[6 + i]) for i, k in enumerate(_TIMINGS)}
    return int(h[1]), GenerationOutput(
        request_id=int(h[2]), prompt_ids=prompt, token_ids=toks, text=tokenizer.decode(toks), finish_reason=reason,
        usage={"prompt_tokens": n_p, "completion_tokens": n_t, "total_tokens": n_p + n_t}, timings=timings)
