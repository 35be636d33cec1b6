"""Broadcast lifecycle rules and the batch sender, free of Django (reference broadcasting/
signals.py:5-48, services.py:240-291, tasks.py:45-148).

Lifecycle: DRAFT -(scheduled_at set)-> SCHEDULED -(due, picked by the beat task)-> SENDING
-(all batches recorded)-> COMPLETED | PARTIAL_FAILURE | FAILED; CANCELED is terminal; clearing
scheduled_at of a SCHEDULED campaign returns it to DRAFT."""
from __future__ import annotations

import logging
from typing import Iterable, Iterator, List, Optional, Sequence, Tuple

from assistant.bot.domain import Answer, MultiPartAnswer, SingleAnswer
from assistant.bot.exceptions import UserUnavailableError

logger = logging.getLogger(__name__)

DRAFT, SCHEDULED, SENDING = "DRAFT", "SCHEDULED", "SENDING"
COMPLETED, PARTIAL_FAILURE, FAILED, CANCELED = "COMPLETED", "PARTIAL_FAILURE", "FAILED", "CANCELED"
STATUSES = (DRAFT, SCHEDULED, SENDING, COMPLETED, PARTIAL_FAILURE, FAILED, CANCELED)
TERMINAL = (COMPLETED, PARTIAL_FAILURE, FAILED, CANCELED)
STAT_FIELDS = frozenset({"status", "started_at", "completed_at", "total_recipients", "successful_sents",
                         "failed_sents", "updated_at"})
BATCH_SIZE = 100


def schedule_transition(status: str, scheduled_at, original_status: Optional[str],
                        update_fields: Optional[Iterable[str]] = None) -> str:
    """Status a campaign should be saved with (the pre_save rule).  Saves that touch only status /
    statistics fields are left alone so the sending machinery never re-triggers it."""
    if update_fields is not None and set(update_fields) <= STAT_FIELDS:
        return status
    if scheduled_at and status == DRAFT:
        return SCHEDULED
    if scheduled_at is None and status == SCHEDULED and (original_status or DRAFT) == SCHEDULED:
        return DRAFT
    return status


def final_status(total: Optional[int], successful: int, failed: int) -> str:
    if not total:
        return COMPLETED
    if failed >= total and successful == 0:
        return FAILED
    if failed > 0:
        return PARTIAL_FAILURE
    return COMPLETED


def batches(chat_ids: Sequence[str], size: int = BATCH_SIZE) -> Iterator[List[str]]:
    for i in range(0, len(chat_ids), size):
        yield list(chat_ids[i:i + size])


def unique_in_order(ids: Iterable[str]) -> List[str]:
    """Distinct chat ids (portable replacement of the reference's PostgreSQL-only DISTINCT ON)."""
    seen, out = set(), []
    for x in ids:
        if x not in seen:
            seen.add(x)
            out.append(x)
    return out


async def post_answer(platform, chat_id: str, answer: Answer) -> None:
    if isinstance(answer, MultiPartAnswer):
        parts = answer.parts
    elif isinstance(answer, SingleAnswer):
        parts = [answer]
    else:
        raise TypeError(f"unsupported answer type {type(answer)}")
    for part in parts:
        await platform.post_answer(chat_id, part)


async def send_batch(platform, chat_ids: Sequence[str], answer: Answer) -> Tuple[int, int, List[str]]:
    """Deliver ``answer`` to every chat sequentially -> (successful, failed, unavailable chat ids)."""
    ok = failed = 0
    unavailable: List[str] = []
    for chat_id in chat_ids:
        try:
            await post_answer(platform, chat_id, answer)
            ok += 1
        except UserUnavailableError as e:
            failed += 1
            unavailable.append(str(e.chat_id or chat_id))
        except Exception:
            logger.exception("broadcast delivery to %s failed", chat_id)
            failed += 1
    return ok, failed, unavailable
