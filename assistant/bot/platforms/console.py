"""Console platform: prints answers (with buttons / reply keyboards) and appends every turn to a JSONL
history file (reference bot/management/commands/chat.py:96-160)."""
from __future__ import annotations

import json
import logging
from typing import List, Optional

from assistant.bot.domain import BotPlatform, MultiPartAnswer, SingleAnswer

logger = logging.getLogger(__name__)


def answer_log_entry(answer: SingleAnswer) -> dict:
    entry = {"role": "assistant", "text": answer.text}
    if answer.buttons:
        entry["buttons"] = [[{"text": b.text, "callback_data": b.callback_data, "url": b.url} for b in row]
                            for row in answer.buttons]
    if answer.reply_keyboard:
        entry["reply_keyboard"] = [[getattr(b, "text", b) for b in row] for row in answer.reply_keyboard]
    return entry


class ConsolePlatform(BotPlatform):
    def __init__(self, history_file: Optional[str] = None, printer=print, log: Optional[List[dict]] = None):
        self.history_file = history_file
        self.printer = printer
        self.log = log if log is not None else []

    @property
    def codename(self) -> str:
        return "console"

    def record(self, entry: dict) -> None:
        self.log.append(entry)
        if self.history_file:
            try:
                with open(self.history_file, "a", encoding="utf-8") as f:
                    f.write(json.dumps(entry, ensure_ascii=False) + "\n")
            except OSError:
                logger.exception("cannot write chat history")

    async def post_answer(self, chat_id: str, answer):
        parts = answer.parts if isinstance(answer, MultiPartAnswer) else [answer]
        for part in parts:
            entry = answer_log_entry(part)
            if self.printer:
                self.printer(f"Bot: {part.text}")
                for row in entry.get("buttons", []):
                    self.printer(" ".join(f"[{b['text']}]({b['callback_data'] or b['url']})" for b in row))
                for row in entry.get("reply_keyboard", []):
                    self.printer(" ".join(f"{{{b}}}" for b in row))
            self.record(entry)

    async def get_update(self, request):
        raise NotImplementedError("console updates are built by the session")

    async def action_typing(self, chat_id):
        return None
