"""One-shot all-reduce over IPC-mapped peer buffers (kernel: csrc/kernels/allreduce.hip).

For the latency-bound all-reduces of TP decode (2 per layer, [batch, hidden] bf16: 16 KB - 2 MB).
Every rank reads all peers directly over xGMI, one hop on all 7 links at once.  RCCL's ring instead
takes 2(W-1) serial steps over 2 of the links.  Larger messages (prefill) fall back to RCCL.

    ar = CustomAllReduce(group, device)      # collective: exchanges IPC handles over `group`
    ar.all_reduce(x)                         # in place; x bf16, contiguous, <= max_bytes
    ar.close()

The buffers come from ``hipExtMallocWithFlags(..., hipDeviceMallocUncached)`` (fine-grained,
uncached: flag and staging accesses are coherent across xGMI, not only at kernel boundaries),
outside the torch caching allocator, so IPC handles cover the whole allocation.  Each rank has one buffer: a signal area plus two staging halves of
``max_bytes``.  The kernel's epochs live on the device, so calls can be captured in HIP graphs.
A peer that never arrives makes the kernel set an error flag instead of hanging, write NaN over
the segments it could not reduce and leave its epoch where it was; the flag is sticky, so every
later call on this rank only poisons its output.  The engine enqueues a copy of the flag behind
every TP step (``enqueue_error_check``) and raises ``CustomAllReduceError`` when it reads it set
after the step's own sync (``raise_if_error``): the step's requests fail (gpu_service answers 500),
the worker turns unhealthy (/health 503) and the launcher restarts the group -- the reference's
"a failed generation is an HTTP 500" (gpu_service/main.py:105-107) for a desynchronised TP group.
``check_error`` is the synchronous form (tests, benchmarks).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ..ops._lib import native, stream


class CustomAllReduceError(RuntimeError):
    pass


class CustomAllReduce:
    def __init__(self, group=None, device=None, max_bytes: int = 8 << 20, spin_limit: int = 1 << 24,
                 exchange_group=None, uncached: bool = True):
        """``group``: the ranks that reduce together.  ``exchange_group``: where the IPC handles
        travel; it defaults to ``group`` and may be a gloo group."""
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if self.world > 8:
            raise ValueError("one-shot all-reduce supports up to 8 ranks (one xGMI node)")
        self.device = torch.device(device if device is not None else "cuda")
        self.max_bytes = int(max_bytes)
        self.spin_limit = int(spin_limit)
        n = native()
        self._n = n
        sig = n.allreduce_signal_bytes()
        with torch.cuda.device(self.device):
            self.base = n.allreduce_buffer_alloc(sig + 2 * self.max_bytes, uncached)
            handle = n.ipc_get_handle(self.base)
            handles = [None] * self.world
            if self.world > 1:
                dist.all_gather_object(handles, handle, group=exchange_group or group)
            else:
                handles = [handle]
            self.bases = [self.base if r == self.rank else n.ipc_open_handle(handles[r]) for r in range(self.world)]
            for b in self.bases:
                n.ipc_probe(b)  # a bad mapping raises here, never inside the kernel
        self._closed = False
        self._exchange = exchange_group or group
        # the error word's host copy (pinned: the async copy never stalls the stream)
        self._err_host = torch.zeros((1,), dtype=torch.int32, pin_memory=True)
        # fault injection (tests): this many of the next calls return without reducing, as a rank
        # that dropped out of the collective would
        self.skip_next = 0
        if self.world > 1:
            dist.barrier(group=self._exchange)

    def eligible(self, x: torch.Tensor) -> bool:
        nb = x.numel() * x.element_size()
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and nb % 16 == 0
                and 0 < nb <= self.max_bytes and x.data_ptr() % 16 == 0)

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        """In-place sum over the group.  Every rank gets bitwise the same result, because the fp32
        sum runs in rank order."""
        if not self.eligible(x):
            raise ValueError("custom all-reduce needs a contiguous bf16 CUDA tensor of <= max_bytes (16-B multiple)")
        if self.skip_next > 0:
            self.skip_next -= 1
            return x
        self._n.custom_allreduce(self.bases, self.rank, x.data_ptr(), x.numel() * 2, self.max_bytes, self.spin_limit,
                                 stream(x))
        return x

    def check_error(self) -> None:
        """Call after a synchronisation point: raises if a peer failed to arrive within the spin limit."""
        if self._n.allreduce_error(self.base, 1):
            raise CustomAllReduceError("custom all-reduce: a peer did not arrive (group broken or desynchronised)")

    def norm_eligible(self, partial: torch.Tensor, cols: int) -> bool:
        """Whether ``all_reduce_rmsnorm`` takes this partial: fp32 slabs [S, rows, cols] or bf16
        [rows, cols], contiguous, whose bf16 rows fit one staging half."""
        if not partial.is_cuda or not partial.is_contiguous() or cols % 8 or cols > 16384:
            return False
        rows = partial.shape[-2]
        ok_dtype = (partial.dtype == torch.float32 and partial.dim() == 3) or \
                   (partial.dtype == torch.bfloat16 and partial.dim() == 2)
        return ok_dtype and partial.shape[-1] == cols and rows * cols * 2 <= self.max_bytes

    def all_reduce_rmsnorm(self, partial: torch.Tensor, residual: torch.Tensor | None, w: torch.Tensor, eps: float):
        """One launch for a TP decode all-reduce site: sums this rank's split-K slabs (or takes its
        bf16 partial), all-reduces over the group, adds the residual and applies the RMSNorm ->
        (normed, new residual).  Bitwise ``slab_reduce`` + ``all_reduce`` + ``ops.rmsnorm``."""
        cols = w.numel()
        if not self.norm_eligible(partial, cols):
            raise ValueError("all_reduce_rmsnorm: fp32 slabs [S, rows, cols] or bf16 [rows, cols] within max_bytes")
        rows = partial.shape[-2]
        out = torch.empty((rows, cols), dtype=torch.bfloat16, device=partial.device)
        res_out = torch.empty_like(out) if residual is not None else None
        if residual is not None and (residual.dtype != torch.bfloat16 or not residual.is_contiguous()
                                     or tuple(residual.shape) != (rows, cols)):
            raise ValueError("residual must be a contiguous bf16 [rows, cols]")
        slabs = partial.dtype == torch.float32
        if self.skip_next > 0:  # fault injection: this rank drops out of the collective
            self.skip_next -= 1
            return out.zero_(), (res_out.zero_() if res_out is not None else None)
        self._n.custom_allreduce_rmsnorm(
            self.bases, self.rank, partial.data_ptr() if slabs else 0, partial.shape[0] if slabs else 0,
            rows * cols if slabs else 0, 0 if slabs else partial.data_ptr(),
            residual.data_ptr() if residual is not None else 0, res_out.data_ptr() if res_out is not None else 0,
            out.data_ptr(), w.data_ptr(), rows, cols, float(eps), self.max_bytes, self.spin_limit, stream(partial))
        return out, res_out

    def enqueue_error_check(self, s: int | None = None) -> None:
        """Copies the error word to the pinned host word behind the work on stream ``s`` (default:
        the current stream).  Read it with ``raise_if_error`` after that stream is synchronised."""
        self._n.allreduce_error_async(self.base, self._err_host.data_ptr(),
                                      torch.cuda.current_stream(self.device).cuda_stream if s is None else s)

    def raise_if_error(self) -> None:
        """After the stream that ran ``enqueue_error_check`` was synchronised: raises if a peer failed
        to arrive in any all-reduce enqueued before it.  The word stays set on the device (sticky)
        until ``reset_error``."""
        if int(self._err_host[0]):
            raise CustomAllReduceError("custom all-reduce: a TP peer did not arrive (group broken or desynchronised); "
                                       "the step's outputs are poisoned")

    def reset_error(self) -> None:
        self._n.allreduce_error(self.base, 1)
        self._err_host.zero_()

    def close(self) -> None:
        """Collective: no rank frees its buffer while a peer's last kernel may still read it."""
        if self._closed:
            return
        self._closed = True
        torch.cuda.synchronize(self.device)
        if self.world > 1 and dist.is_initialized():
            dist.barrier(group=self._exchange)
        for r, b in enumerate(self.bases):
            if r != self.rank:
                self._n.ipc_close_handle(b)
        self._n.allreduce_buffer_free(self.base)


def maybe_create(group, device, world: int):
    """The TP all-reduce for the model.  None (-> RCCL) when disabled (``DAB_CUSTOM_AR=0``), on one
    rank, or when IPC mapping fails (e.g. ranks on different nodes)."""
    if world <= 1 or os.environ.get("DAB_CUSTOM_AR", "1") == "0" or not torch.cuda.is_available():
        return None
    try:
        return CustomAllReduce(group, device)
    except Exception as exc:  # pragma: no cover - depends on the runtime
        import logging

        logging.getLogger(__name__).warning("custom all-reduce unavailable (%s); using RCCL", exc)
        return None
