"""Tensor-parallel serving control plane: one leader, lock-step followers.

A TP generator (Llama-3-70B over 8 GPUs) is one engine spread over a group of processes.  Every rank
must run the same scheduler steps with the same requests, because each forward contains the group's
all-reduces.  The HTTP-facing rank (the leader, TP rank 0) owns the request stream.  The other ranks
follow:

* ``TPLeader`` wraps the leader's ``LLMEngine`` with the same API (``add_request`` / ``step`` /
  ``abort`` / ``pop_output`` ...).  Adds and aborts are queued and shipped with the next ``step``
  command, so the control traffic is one small broadcast per engine step.
* ``follow(engine, group)`` is the loop the other ranks run: receive a command, apply it to the
  local engine, step.  Sampled tokens are already identical on all ranks, because the engine
  broadcasts TP rank 0's tokens inside every step.

The control messages go over a gloo group as fixed-shape int64 tensors (``parallel/wire.py``: one
header table + payload per step, no pickles), independent of the RCCL data plane.  The leader can
therefore sit in an asyncio server thread without touching the GPU collectives.

    leader = TPLeader(engine, ctrl_group)        # rank 0: hand to LLMWorker / gpu_service
    follow(engine, ctrl_group)                   # ranks 1..N-1: blocks until leader.shutdown()
"""
from __future__ import annotations

import torch.distributed as dist

from . import wire


def control_group(ranks: list[int] | None = None, timeout_s: float = 30 * 24 * 3600):
    """A gloo group over the TP ranks for host-side control messages (None: the whole world).  The
    timeout is long because followers legitimately wait as long as the service is idle."""
    import datetime

    return dist.new_group(ranks, backend="gloo", timeout=datetime.timedelta(seconds=timeout_s))


def _src(group) -> int:
    return dist.get_global_rank(group, 0) if group is not None else 0


class TPLeader:
    def __init__(self, engine, group=None):
        self.engine = engine
        self.group = group
        self._pending: list = []  # wire ADD / ABORT items of the next step
        self._stopped = False
        engine.auto_expire = False  # deadlines are decided here and mirrored as aborts

    # ---- engine API used by LLMWorker / RAGPipeline / gpu_service
    def add_request(self, prompt_ids, params=None, request_id=None) -> int:
        rid = self.engine.add_request(prompt_ids, params, request_id)
        r = self.engine.waiting[-1]  # the request just queued: ship the normalised prompt + params
        self._pending.append(wire.add_item(0, rid, list(r.prompt), r.params))
        return rid

    def abort(self, rid: int, reason: str = "abort") -> bool:
        self._pending.append(wire.abort_item(0, rid, reason))
        return self.engine.abort(rid, reason)

    def step(self) -> list[int]:
        for rid in self.engine.expired():
            self.abort(rid, "timeout")
        self._send(self._pending + [wire.item([wire.STEP, 0])])
        self._pending = []
        return self.engine.step()

    def fail_all(self) -> list[int]:
        self._send([wire.item([wire.FAIL, 0])])
        self._pending = []
        return self.engine.fail_all()

    def shutdown(self) -> None:
        if not self._stopped:
            self._stopped = True
            self._send([wire.item([wire.STOP])])

    def _send(self, items) -> None:
        wire.bcast_batch(items, _src(self.group), self.group)

    def __getattr__(self, name):  # read-only state (stats, tokenizer, finished, has_unfinished ...)
        return getattr(self.engine, name)


def follow(engine, group=None) -> int:
    """Follower loop: mirrors the leader's commands on the local engine until STOP.  Returns the
    number of steps run."""
    steps = 0
    engine.auto_expire = False
    while True:
        stepping = False
        for h, p in wire.bcast_batch(None, _src(group), group):
            k = int(h[0])
            if k == wire.STOP:
                return steps
            if k == wire.FAIL:
                engine.fail_all()
            elif k == wire.ADD:
                _, rid, prompt, params = wire.read_add(h, p)
                engine.add_request(prompt, params, request_id=rid)
            elif k == wire.ABORT:
                _, rid, reason = wire.read_abort(h, p)
                if engine.abort(rid, reason):
                    engine.pop_output(rid)
            elif k == wire.STEP:
                stepping = True
        if stepping:
            for rid in engine.step():
                engine.pop_output(rid)  # outputs are served by the leader only
            steps += 1
