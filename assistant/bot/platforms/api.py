"""In-process platform for the REST API and the console: answers are collected instead of sent."""
from __future__ import annotations

from typing import List, Tuple

from assistant.bot.domain import BotPlatform, SingleAnswer, Update


class CollectingPlatform(BotPlatform):
    def __init__(self, codename: str = "api"):
        self._codename = codename
        self.sent: List[Tuple[str, SingleAnswer]] = []
        self.typing_calls = 0

    @property
    def codename(self) -> str:
        return self._codename

    async def get_update(self, request) -> Update:
        data = getattr(request, "data", request)
        return Update.from_dict(data)

    async def post_answer(self, chat_id: str, answer: SingleAnswer):
        self.sent.append((chat_id, answer))

    async def action_typing(self, chat_id):
        self.typing_calls += 1
