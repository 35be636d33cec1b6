"""Broadcast lifecycle rules and batch sending without Django (reference broadcasting/signals.py,
services.py:240-291, tasks.py:45-148)."""
import asyncio
import datetime as dt

from assistant.bot.domain import MultiPartAnswer, SingleAnswer
from assistant.bot.exceptions import UserUnavailableError
from assistant.bot.platforms.api import CollectingPlatform
from assistant.broadcasting import core


def test_schedule_transition():
    now = dt.datetime(2026, 1, 1)
    assert core.schedule_transition(core.DRAFT, now, None) == core.SCHEDULED
    assert core.schedule_transition(core.SCHEDULED, None, core.SCHEDULED) == core.DRAFT
    assert core.schedule_transition(core.SCHEDULED, None, None) == core.SCHEDULED  # new instance
    assert core.schedule_transition(core.SENDING, None, core.SENDING) == core.SENDING
    assert core.schedule_transition(core.DRAFT, now, None, update_fields=["status", "started_at"]) == core.DRAFT
    assert core.schedule_transition(core.DRAFT, now, None, update_fields=["scheduled_at"]) == core.SCHEDULED


def test_final_status_and_batches():
    assert core.final_status(0, 0, 0) == core.COMPLETED
    assert core.final_status(None, 0, 0) == core.COMPLETED
    assert core.final_status(10, 10, 0) == core.COMPLETED
    assert core.final_status(10, 7, 3) == core.PARTIAL_FAILURE
    assert core.final_status(10, 0, 10) == core.FAILED
    ids = [str(i) for i in range(250)]
    assert [len(b) for b in core.batches(ids)] == [100, 100, 50]
    assert core.unique_in_order(["a", "b", "a", "c", "b"]) == ["a", "b", "c"]


def test_send_batch_counts_and_unavailable():
    class Flaky(CollectingPlatform):
        async def post_answer(self, chat_id, answer):
            if chat_id == "blocked":
                raise UserUnavailableError(chat_id)
            if chat_id == "broken":
                raise RuntimeError("network")
            await super().post_answer(chat_id, answer)

    p = Flaky()
    ok, failed, unavailable = asyncio.run(core.send_batch(p, ["a", "blocked", "b", "broken"], SingleAnswer("hi")))
    assert (ok, failed, unavailable) == (2, 2, ["blocked"])
    assert [c for c, _ in p.sent] == ["a", "b"]
    p2 = CollectingPlatform()
    multi = MultiPartAnswer([SingleAnswer("1"), SingleAnswer("2")])
    assert asyncio.run(core.send_batch(p2, ["x"], multi)) == (1, 0, [])
    assert [a.text for _, a in p2.sent] == ["1", "2"]
