"""AI domain types (reference ai/domain.py:5-30)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, TypedDict, Union


@dataclass
class AIResponse:
    result: Union[str, Dict]  # text, or a dict in JSON mode
    usage: Dict = None
    length_limited: bool = False

    @property
    def model(self):
        return self.usage.get("model") if self.usage else None


class _MessageBase(TypedDict):
    role: str
    content: str


class Message(_MessageBase, total=False):
    images: List[str]  # base64 JPEG payloads (multimodal providers)


def user_message(content: str) -> Message:
    return Message(role="user", content=content)


def assistant_message(content: str) -> Message:
    return Message(role="assistant", content=content)


def system_message(content: str) -> Message:
    return Message(role="system", content=content)
