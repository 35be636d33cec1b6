"""Context assembly within the token budget (reference steps/fill_info.py:6-33)."""
from assistant.utils.sync import sync_to_async

from assistant.bot.services.context_service.steps.base import ContextProcessingStep


class FillInfoStep(ContextProcessingStep):
    max_tokens_share = 0.15
    max_documents = 3

    async def run(self):
        await sync_to_async(self._run_sync)()

    def _run_sync(self):
        documents = list(self._state.documents or [])
        if not documents:
            return
        budget = int(self._fast_ai.context_size * self.max_tokens_share)
        output, n = "", 0
        for document in documents[: self.max_documents]:
            path = document.wiki.path if document.wiki_id else document.name
            candidate = f"{output}# {path}:\n```\n{document.content}\n```\n"
            if output and self._fast_ai.calculate_tokens(candidate) > budget:
                break
            output, n = candidate, n + 1
        self._logger.info("filled %d documents (%d tokens)", n, self._fast_ai.calculate_tokens(output))
        self._state.documents = self._state.documents[:n]
        self._state.final_info = output
        self._state.context_is_ok = True
