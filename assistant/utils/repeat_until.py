"""LLM output-validation loops (reference utils/repeat_until.py:6-54).

``MaxAttemptsExceededError`` lives here (the reference imported it upward from assistant.bot.utils,
which made the utilities depend on the Telegram platform); assistant.bot.utils re-exports it.
"""
from __future__ import annotations

import logging
from typing import Any, Awaitable, Callable

logger = logging.getLogger(__name__)


class MaxAttemptsExceededError(Exception):
    """A validated call did not produce an acceptable result within its attempt budget."""


async def repeat_until(func: Callable[..., Awaitable[Any]], *args: Any, max_attempts: int = 5,
                       condition: Callable[[Any], bool], **kwargs: Any) -> Any:
    """Call ``await func(*args, **kwargs)`` until ``condition(result)`` holds; raise after ``max_attempts``."""
    for attempt in range(1, max_attempts + 1):
        result = await func(*args, **kwargs)
        try:
            ok = condition(result)
        except Exception as exc:  # a condition that crashes on malformed output counts as a miss
            logger.debug("condition raised %r", exc)
            ok = False
        if ok:
            return result
        logger.warning("attempt %d/%d rejected: %r", attempt, max_attempts, result)
    raise MaxAttemptsExceededError(f"condition not met after {max_attempts} attempts")


async def retry_call(func: Callable[..., Awaitable[Any]], *args: Any, max_attempts: int = 5, **kwargs: Any) -> Any:
    """Call until it does not raise; the last error is chained into ``MaxAttemptsExceededError``."""
    last: Exception | None = None
    for attempt in range(1, max_attempts + 1):
        try:
            return await func(*args, **kwargs)
        except Exception as exc:
            last = exc
            logger.warning("attempt %d/%d failed: %s", attempt, max_attempts, exc)
    raise MaxAttemptsExceededError(f"call failed after {max_attempts} attempts") from last
