"""Access to the native extension and small launch helpers.

Dispatch rule used by every op in this package: a tensor on the GPU runs the hand-written gfx950
kernel from ``_native`` (and raises if the extension is missing -- there is no silent eager
fallback on a GPU), a CPU tensor runs the plain-PyTorch fp32 reference from
``ops/reference.py`` (the numerics oracle used by the CPU test-suite).
"""
from __future__ import annotations

import importlib
import os

import torch

_native = None


class NativeExtensionMissing(RuntimeError):
    pass


def native():
    """The compiled ``_native`` module; builds it in-tree on first use if allowed."""
    global _native
    if _native is None:
        try:
            _native = importlib.import_module("django_assistant_bot_amd._native")
        except ImportError as exc:
            if os.environ.get("DAB_AUTOBUILD", "1") == "1":
                from django_assistant_bot_amd.build import build

                build()
                _native = importlib.import_module("django_assistant_bot_amd._native")
            else:
                raise NativeExtensionMissing(
                    "django_assistant_bot_amd._native is not built: run `python -m django_assistant_bot_amd.build`"
                ) from exc
    return _native


def has_native() -> bool:
    try:
        native()
        return True
    except Exception:
        return False


def ptr(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.data_ptr()


def stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def expect(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)


def expect_bf16_contig(*ts: torch.Tensor | None) -> None:
    for t in ts:
        if t is None:
            continue
        if t.dtype != torch.bfloat16:
            raise TypeError(f"expected bfloat16 tensor, got {t.dtype}")
        if not t.is_contiguous():
            raise ValueError("expected a contiguous tensor")


def same_device(*ts: torch.Tensor | None) -> None:
    devs = {t.device for t in ts if t is not None}
    if len(devs) > 1:
        raise ValueError(f"tensors on different devices: {devs}")
