"""Mutable state shared by the context pipeline steps (reference context_service/state.py)."""
from __future__ import annotations

from typing import List, Optional


class ContextProcessingState:
    def __init__(self):
        self.messages: Optional[List[dict]] = None
        self.topic = None  # WikiDocument (root topic) or None for small talk
        self.related_questions: list = []
        self.documents: list = []
        self.final_info: Optional[str] = None
        self.context_is_ok: Optional[bool] = None
        self.done: bool = False

    @property
    def user_question(self) -> str:
        return (self.messages[-1]["content"] or "").strip()

    @user_question.setter
    def user_question(self, value: str):
        self.messages[-1] = dict(self.messages[-1], content=value)
