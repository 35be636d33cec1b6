"""Campaign services (reference broadcasting/services.py:21-291).

initiate_campaign_sending: under a row lock SCHEDULED -> SENDING, resolve recipients (every available
instance of the bot, distinct users -- portable, no PostgreSQL DISTINCT ON), record the total, then fan
out ``send_broadcast_batch`` tasks of 100 chats.  record_batch_results adds a batch's counts atomically
and triggers finalize when all recipients are accounted for; finalize_campaign sets the final status.
"""
from __future__ import annotations

import logging
from typing import List

from django.db import transaction
from django.db.models import F
from django.utils import timezone

from assistant.bot.models import Instance
from assistant.broadcasting import core
from assistant.utils.sync import sync_to_async

from .models import BroadcastCampaign

logger = logging.getLogger(__name__)


def resolve_target_chat_ids(campaign: BroadcastCampaign) -> List[str]:
    ids = (Instance.objects.filter(bot=campaign.bot, is_unavailable=False, user__platform=campaign.platform)
           .order_by("user__user_id").values_list("user__user_id", flat=True))
    return core.unique_in_order(ids)


async def schedule_campaign_sending(campaign: BroadcastCampaign) -> bool:
    """DRAFT -> SCHEDULED (a missing or past scheduled_at means: pick up on the next beat)."""
    if campaign.status != BroadcastCampaign.Status.DRAFT:
        logger.warning("campaign %s is %s, not DRAFT; not scheduling", campaign.id, campaign.status)
        return False
    campaign.status = BroadcastCampaign.Status.SCHEDULED
    await sync_to_async(campaign.save)(update_fields=["status"])
    return True


def _begin_sending(campaign_id: int):
    with transaction.atomic():
        c = BroadcastCampaign.objects.select_for_update().select_related("bot").filter(id=campaign_id).first()
        if c is None or c.status != BroadcastCampaign.Status.SCHEDULED:
            return None, []
        chat_ids = resolve_target_chat_ids(c)
        c.status = BroadcastCampaign.Status.SENDING
        c.started_at = timezone.now()
        c.total_recipients = len(chat_ids)
        c.save(update_fields=["status", "started_at", "total_recipients"])
        return c, chat_ids


async def initiate_campaign_sending(campaign_id: int) -> int:
    """Returns the number of dispatched batches."""
    try:
        campaign, chat_ids = await sync_to_async(_begin_sending)(campaign_id)
        if campaign is None:
            logger.warning("campaign %s not found or not SCHEDULED", campaign_id)
            return 0
        if not chat_ids:
            await finalize_campaign(campaign_id)
            return 0
        from .tasks import send_broadcast_batch

        n = 0
        for batch in core.batches(chat_ids):
            send_broadcast_batch.delay(campaign_id=campaign.id, bot_codename=campaign.bot.codename,
                                       platform_codename=campaign.platform, chat_ids=batch,
                                       message_content_data=campaign.message())
            n += 1
        logger.info("campaign %s: %d recipients in %d batches", campaign_id, len(chat_ids), n)
        return n
    except Exception:
        logger.exception("campaign %s initiation failed", campaign_id)
        await sync_to_async(BroadcastCampaign.objects.filter(id=campaign_id).update)(
            status=BroadcastCampaign.Status.FAILED, completed_at=timezone.now())
        return 0


def record_batch_results_sync(campaign_id: int, successful: int, failed: int) -> bool:
    """Atomic counter update; returns True when the campaign is complete (finalize triggered)."""
    with transaction.atomic():
        updated = BroadcastCampaign.objects.filter(id=campaign_id, status=BroadcastCampaign.Status.SENDING).update(
            successful_sents=F("successful_sents") + successful, failed_sents=F("failed_sents") + failed,
            updated_at=timezone.now())
        if not updated:
            logger.warning("campaign %s not SENDING; batch results ignored", campaign_id)
            return False
        c = BroadcastCampaign.objects.get(id=campaign_id)
        done = c.total_recipients is not None and c.successful_sents + c.failed_sents >= c.total_recipients
    if done:
        from .tasks import finalize_campaign_task
        transaction.on_commit(lambda: finalize_campaign_task.delay(campaign_id))
    return done


record_batch_results = sync_to_async(record_batch_results_sync)


def finalize_campaign_sync(campaign_id: int) -> bool:
    with transaction.atomic():
        c = BroadcastCampaign.objects.select_for_update().filter(id=campaign_id).first()
        if c is None:
            return False
        if c.status != BroadcastCampaign.Status.SENDING:
            if c.status == BroadcastCampaign.Status.FAILED and c.completed_at is None:
                c.completed_at = c.started_at or timezone.now()
                c.save(update_fields=["completed_at"])
            return c.status in core.TERMINAL
        c.status = core.final_status(c.total_recipients, c.successful_sents, c.failed_sents)
        c.completed_at = timezone.now()
        c.save(update_fields=["status", "completed_at", "updated_at"])
        logger.info("campaign %s finalized: %s", campaign_id, c.status)
        return True


finalize_campaign = sync_to_async(finalize_campaign_sync)
