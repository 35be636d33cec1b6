"""Offline-tuned vendor GEMM solutions (PyTorch TunableOp results, tuned on MI355X by
``benchmarks/tune_gemms.py`` with cold-cache rotating buffers and filtered to clear winners).

TunableOp is NOT enabled globally: with it on, every untuned shape would go through TunableOp's
"Default" path, which measured slower than torch's normal dispatch for several decode shapes.  Only
GEMMs whose exact (M, N, K) is in a loaded file are dispatched through it; everything else keeps
the library heuristic.
"""
from __future__ import annotations

import logging
import os
from typing import Set, Tuple

import torch
import torch.nn.functional as F

logger = logging.getLogger(__name__)

TUNING_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning")
_TUNED: Set[Tuple[int, int, int]] = set()
_LOADED: Set[str] = set()


def tuning_file(model: str, tp: int, arch: str) -> str:
    return os.path.join(TUNING_DIR, f"tunableop_{model}_tp{tp}_{arch}.csv")


def load(path: str) -> int:
    """Load a TunableOp results file; returns the number of tuned shapes (0 if absent/rejected)."""
    if path in _LOADED:
        return len(_TUNED)
    if not os.path.exists(path) or not torch.cuda.is_available():
        return 0
    import torch.cuda.tunable as tn

    shapes = set()
    with open(path) as f:
        for line in f:
            parts = line.strip().split(",")
            if len(parts) >= 3 and parts[0].startswith("GemmTunableOp") and parts[1].startswith("tn_"):
                n, m, k = (int(v) for v in parts[1].split("_")[1:4])
                shapes.add((m, n, k))
    try:
        ok = tn.read_file(path)
    except Exception as e:  # validator mismatch (other torch / hipBLASLt build): keep heuristics
        logger.warning("GEMM tuning file %s rejected: %s", path, e)
        return 0
    if ok is False:
        return 0
    tn.tuning_enable(False)
    _TUNED.update(shapes)
    _LOADED.add(path)
    logger.info("loaded %d tuned GEMM shapes from %s", len(shapes), path)
    return len(shapes)


def is_tuned(m: int, n: int, k: int) -> bool:
    return (m, n, k) in _TUNED


def linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """F.linear that uses the tuned solution when this exact shape has one."""
    if _TUNED and x.is_cuda and x.dim() == 2 and (x.shape[0], w.shape[0], w.shape[1]) in _TUNED:
        import torch.cuda.tunable as tn

        tn.enable(True)
        try:
            return F.linear(x, w)
        finally:
            tn.enable(False)
    return F.linear(x, w)
