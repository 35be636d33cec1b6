"""RAG context pipeline (reference bot/services/context_service/service.py:19-83).

Default pipeline:  [ClassifyStep || EmbeddingsStep] -> InterruptIfSmallTalk -> ChooseKnownQuestion ->
FillInfo -> FinalPrompt.  Steps in a list run concurrently; after every stage the pipeline stops if
``do_interrupt()`` (a newer user message arrived) or ``state.done`` (small talk) is set.  Subclasses
can override ``pipeline`` to enable the optional steps (ReformulateQuestion, ChooseDocs, CheckContext).
"""
from __future__ import annotations

import asyncio
import logging
from typing import Awaitable, Callable, Dict, List, Type, Union

from assistant.bot.services.context_service.state import ContextProcessingState
from assistant.bot.services.context_service.steps.base import ContextProcessingStep
from assistant.bot.services.context_service.steps.choose_known_question import ChooseKnownQuestionStep
from assistant.bot.services.context_service.steps.classify import ClassifyStep
from assistant.bot.services.context_service.steps.embeddings import EmbeddingsStep
from assistant.bot.services.context_service.steps.fill_info import FillInfoStep
from assistant.bot.services.context_service.steps.final_prompt import FinalPromptStep
from assistant.bot.services.context_service.steps.interruptions import InterruptIfSmallTalkStep

logger = logging.getLogger(__name__)

Stage = Union[Type[ContextProcessingStep], List[Type[ContextProcessingStep]]]


class ContextService:
    pipeline: List[Stage] = [
        [ClassifyStep, EmbeddingsStep],
        InterruptIfSmallTalkStep,
        ChooseKnownQuestionStep,
        FillInfoStep,
        FinalPromptStep,
    ]

    def __init__(self, bot, fast_ai_model: str, strong_ai_model: str, messages: List[dict],
                 debug_info: Dict = None, do_interrupt: Callable[..., Awaitable[bool]] = None):
        self._bot = bot
        self._fast_ai_model = fast_ai_model
        self._strong_ai_model = strong_ai_model
        self._debug_info = debug_info if debug_info is not None else {}
        self._do_interrupt = do_interrupt
        self._state = ContextProcessingState()
        self._state.messages = list(messages)

    @property
    def state(self) -> ContextProcessingState:
        return self._state

    async def enrich(self) -> List[dict]:
        await self._pipeline(self.pipeline)
        return self._state.messages

    async def _pipeline(self, pipeline: List[Stage]):
        for stage in pipeline:
            await self._run_steps(stage if isinstance(stage, list) else [stage])
            if self._do_interrupt and await self._do_interrupt():
                logger.info("context pipeline interrupted")
                break
            if self._state.done:
                break

    async def _run_steps(self, step_classes):
        steps = [cls(bot=self._bot, state=self._state, fast_ai_model=self._fast_ai_model,
                     strong_ai_model=self._strong_ai_model, debug_info=self._debug_info) for cls in step_classes]
        await asyncio.gather(*(s.run() for s in steps))
