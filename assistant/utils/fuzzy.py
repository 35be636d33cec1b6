"""Fuzzy string matching (the reference used fuzzywuzzy ``process.extractBests`` / ``WRatio``);
stdlib difflib implementation of a weighted ratio: plain, partial and token-sort ratios, 0-100."""
from __future__ import annotations

import re
from difflib import SequenceMatcher

_WS = re.compile(r"\W+", re.UNICODE)


def _norm(s: str) -> str:
    return " ".join(_WS.sub(" ", (s or "").lower()).split())


def ratio(a: str, b: str) -> int:
    return int(round(100 * SequenceMatcher(None, a, b).ratio()))


def partial_ratio(a: str, b: str) -> int:
    short, long_ = (a, b) if len(a) <= len(b) else (b, a)
    if not short:
        return 0
    best = 0
    for blk in SequenceMatcher(None, short, long_).get_matching_blocks():
        start = max(0, blk.b - blk.a)
        best = max(best, ratio(short, long_[start:start + len(short)]))
        if best == 100:
            break
    return best


def token_sort_ratio(a: str, b: str) -> int:
    return ratio(" ".join(sorted(a.split())), " ".join(sorted(b.split())))


def weighted_ratio(a: str, b: str) -> int:
    a, b = _norm(a), _norm(b)
    if not a or not b:
        return 0
    base = ratio(a, b)
    scale = 0.9 if max(len(a), len(b)) / max(1, min(len(a), len(b))) >= 1.5 else 1.0
    return int(round(max(base, partial_ratio(a, b) * scale, token_sort_ratio(a, b) * 0.95)))


def extract_bests(query: str, choices: list, limit: int = 5, score_cutoff: int = 0) -> list:
    """[(choice, score)] best first (stable for equal scores)."""
    scored = [(c, weighted_ratio(query, c)) for c in choices]
    scored = [x for x in scored if x[1] >= score_cutoff]
    scored.sort(key=lambda x: -x[1])
    return scored[:limit]
