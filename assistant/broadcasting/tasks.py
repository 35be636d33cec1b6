"""Broadcast Celery tasks on the ``broadcasting`` queue (reference broadcasting/tasks.py:45-231).
The beat task ``broadcasting.check_scheduled_broadcasts`` starts due campaigns every minute."""
from __future__ import annotations

import logging
from typing import Dict, List

from assistant.assistant.queue import CeleryQueues
from assistant.broadcasting import core
from assistant.utils.sync import async_to_sync, sync_to_async
from assistant.utils.tasks import shared_task

logger = logging.getLogger(__name__)
Q = CeleryQueues.BROADCASTING.value


@shared_task(queue=Q)
def send_broadcast_batch(campaign_id: int, bot_codename: str, platform_codename: str, chat_ids: List[str],
                         message_content_data: Dict):
    return async_to_sync(_send_broadcast_batch_async)(campaign_id, bot_codename, platform_codename, chat_ids,
                                                      message_content_data)


async def _send_broadcast_batch_async(campaign_id, bot_codename, platform_codename, chat_ids, message_content_data):
    from assistant.bot.domain import answer_from_dict
    from assistant.bot.utils import get_bot_platform

    try:
        platform = await sync_to_async(get_bot_platform)(bot_codename, platform_codename)
        answer = answer_from_dict(message_content_data)
        if platform is None:
            raise RuntimeError(f"no platform {platform_codename} for bot {bot_codename}")
    except Exception:
        logger.exception("campaign %s: cannot prepare batch; counting it failed", campaign_id)
        record_batch_results_task.delay(campaign_id, 0, len(chat_ids))
        return
    ok, failed, unavailable = await core.send_batch(platform, chat_ids, answer)
    if unavailable:
        await sync_to_async(mark_users_unavailable)(bot_codename, platform_codename, unavailable)
    record_batch_results_task.delay(campaign_id, ok, failed)


def mark_users_unavailable(bot_codename: str, platform_codename: str, user_ids: List[str]) -> int:
    from assistant.bot.models import Instance

    return Instance.objects.filter(bot__codename=bot_codename, user__platform=platform_codename,
                                   user__user_id__in=user_ids, is_unavailable=False).update(is_unavailable=True)


@shared_task(name="broadcasting.check_scheduled_broadcasts", queue=Q)
def check_scheduled_broadcasts():
    from django.utils import timezone

    from .models import BroadcastCampaign

    due = list(BroadcastCampaign.objects.filter(status=BroadcastCampaign.Status.SCHEDULED,
                                                scheduled_at__lte=timezone.now()).values_list("id", flat=True))
    due += list(BroadcastCampaign.objects.filter(status=BroadcastCampaign.Status.SCHEDULED,
                                                 scheduled_at__isnull=True).values_list("id", flat=True))
    for cid in due:
        start_campaign_sending_task.delay(cid)
    return len(due)


@shared_task(queue=Q)
def start_campaign_sending_task(campaign_id: int):
    from .services import initiate_campaign_sending
    return async_to_sync(initiate_campaign_sending)(campaign_id)


@shared_task(queue=Q)
def record_batch_results_task(campaign_id: int, successful: int, failed: int):
    from .services import record_batch_results_sync
    return record_batch_results_sync(campaign_id, successful, failed)


@shared_task(queue=Q)
def finalize_campaign_task(campaign_id: int):
    from .services import finalize_campaign_sync
    return finalize_campaign_sync(campaign_id)
