"""Ingest helpers (reference processing/utils.py): prompt schemas, newline-bounded text parts, and
the language rule of the validation loops."""
from __future__ import annotations

import os
import re
from typing import Iterable, List, Optional

from assistant.conf import settings
from assistant.utils.json_schema import JSONSchema
from assistant.utils.language import get_language

SCHEMA_DIR = os.path.join(os.path.dirname(os.path.realpath(__file__)), "schemas")
_json_schema = JSONSchema(SCHEMA_DIR)


def json_prompt(name: str, *args, **kwargs) -> str:
    return _json_schema.get_prompt(name, *args, **kwargs)


def split_text_by_parts(text: str, max_part_length: int) -> List[str]:
    """Split on newlines so that every part stays within ``max_part_length`` characters (a single
    longer line becomes its own part).  Unlike the reference, no empty first part is emitted."""
    parts, part = [], ""
    for line in text.splitlines():
        if part and len(part) + len(line) > max_part_length:
            parts.append(part)
            part = ""
        part += line + "\n"
    if part:
        parts.append(part)
    return parts


def estimated_min_length(text: str) -> int:
    """Lower bound on the summed length of an extraction of ``text`` (reference sentences.py:116)."""
    words = len(re.findall(r"\w+", text))
    return min(words * 5, int(len(text.strip()) * 0.8))


def expected_language(source: str) -> Optional[str]:
    """Language LLM outputs must be in: ``settings.PROCESSING_LANGUAGE`` if set, else the language of
    the source text.  (The reference hard-coded 'ru' in every check)"""
    forced = settings.get("PROCESSING_LANGUAGE")
    if forced:
        return forced
    lang = get_language(source or "")
    return lang if lang and lang != "unknown" else None


def language_ok(texts: Iterable[str], expected: Optional[str]) -> bool:
    if not expected:
        return True
    return all(get_language(t) == expected for t in texts if t and t.strip())
