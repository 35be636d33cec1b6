"""Answer orchestration shared by the Celery tasks, the REST API and the console commands
(reference bot/tasks.py:22-129), written against ``BotStore`` so it runs without Django.

``answer_update``: under the per-instance lock, notify a brand-new instance, let the bot handle the
update, then deliver every part of the answer and record it; a ``UserUnavailableError`` from the
platform marks the instance unavailable (broadcasts then skip it)."""
from __future__ import annotations

import logging
from contextlib import asynccontextmanager
from typing import Optional

from assistant.bot.domain import Answer, BotPlatform, MultiPartAnswer, Update
from assistant.bot.exceptions import UserUnavailableError

logger = logging.getLogger(__name__)


@asynccontextmanager
async def _no_lock():
    yield


async def post_answer(platform: BotPlatform, chat_id: str, answer: Answer) -> None:
    parts = answer.parts if isinstance(answer, MultiPartAnswer) else [answer]
    for part in parts:
        await platform.post_answer(chat_id, part)


async def mark_unavailable(store, instance) -> None:
    instance.is_unavailable = True
    await store.save_instance(instance, ["is_unavailable"])


async def answer_update(bot, platform: BotPlatform, update: Update, lock=None,
                        instance_is_new: bool = False) -> Optional[Answer]:
    """Handle one update end to end; returns the delivered answer (or None)."""
    async with (lock if lock is not None else _no_lock()):
        if instance_is_new:
            await bot.on_instance_created()
        answer = await bot.handle_update(update)
    if not answer:
        return None
    try:
        await post_answer(platform, update.chat_id, answer)
        await bot.on_answer_sent(answer)
    except UserUnavailableError as e:
        logger.warning("User %s unavailable; marking instance %s", e.chat_id, bot.instance.id)
        await mark_unavailable(bot.store, bot.instance)
    except Exception:
        logger.exception("Error while sending answer")
    return answer
