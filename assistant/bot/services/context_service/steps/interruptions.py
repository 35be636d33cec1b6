from assistant.bot.services.context_service.steps.base import ContextProcessingStep


class InterruptIfSmallTalkStep(ContextProcessingStep):
    """No knowledge-base context is needed for small talk (reference steps/interruptions.py)."""

    async def run(self):
        if self._state.topic is None:
            self._state.done = True
