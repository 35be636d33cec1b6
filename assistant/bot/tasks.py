"""Celery tasks of the conversation layer (reference bot/tasks.py:21-129).

``answer_task`` answers one update (enqueued by the webhook view / REST API); ``send_answer_task``
delivers a pre-built answer (used by broadcasting and admin tools) unless the user is known to be
unavailable.  The orchestration lives in ``services.answer_service`` (Django-free)."""
from __future__ import annotations

import logging
from typing import Dict

from assistant.assistant.queue import CeleryQueues
from assistant.bot.domain import Update, answer_from_dict
from assistant.bot.exceptions import UserUnavailableError
from assistant.bot.services.answer_service import answer_update, post_answer
from assistant.utils.sync import async_to_sync, sync_to_async
from assistant.utils.tasks import shared_task

logger = logging.getLogger(__name__)


@shared_task(queue=CeleryQueues.QUERY.value)
def answer_task(*args, **kwargs):
    return async_to_sync(_answer_task)(*args, **kwargs)


async def _answer_task(bot_codename: str, dialog_id, platform_codename: str, update: Dict):
    from assistant.bot.models import Dialog, Message
    from assistant.bot.services.instance_service import InstanceLockAsync
    from assistant.bot.store import DjangoBotStore
    from assistant.bot.utils import get_bot_class, get_bot_platform

    update = Update.from_dict(update)
    platform = await sync_to_async(get_bot_platform)(bot_codename, platform_codename)
    dialog = await sync_to_async(
        lambda: Dialog.objects.select_related("instance", "instance__bot", "instance__user").get(id=dialog_id))()
    bot = get_bot_class(bot_codename)(dialog=dialog, platform=platform, store=DjangoBotStore())
    n_messages = await sync_to_async(
        lambda: Message.objects.filter(dialog__instance_id=dialog.instance_id)[:2].count())()
    return await answer_update(bot, platform, update, lock=InstanceLockAsync(dialog.instance),
                               instance_is_new=n_messages <= 1)


@shared_task(queue=CeleryQueues.QUERY.value)
def send_answer_task(*args, **kwargs):
    return async_to_sync(_send_answer_task)(*args, **kwargs)


async def _send_answer_task(bot_codename: str, platform_codename: str, chat_id: str, answer_data: Dict):
    from assistant.bot.models import Instance
    from assistant.bot.utils import get_bot_platform

    instance = await sync_to_async(
        lambda: Instance.objects.filter(bot__codename=bot_codename, user__user_id=chat_id,
                                        user__platform=platform_codename).first())()
    if instance is not None and instance.is_unavailable:
        logger.info("Skipping unavailable user %s (instance %s)", chat_id, instance.id)
        return
    platform = await sync_to_async(get_bot_platform)(bot_codename, platform_codename)
    try:
        answer = answer_from_dict(answer_data)
    except Exception:
        logger.exception("Cannot deserialize answer for %s", chat_id)
        return
    try:
        await post_answer(platform, chat_id, answer)
    except UserUnavailableError:
        if instance is not None:
            instance.is_unavailable = True
            await sync_to_async(instance.save)(update_fields=["is_unavailable"])
    except Exception:
        logger.exception("Error while sending answer to %s", chat_id)
