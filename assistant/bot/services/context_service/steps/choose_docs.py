"""Optional: let the fast model pick up to 3 documents by title (reference steps/choose_docs.py:13-199).
Titles returned by the model are matched back with a fuzzy ratio >= 90."""
from __future__ import annotations

from typing import List, Optional

from assistant.utils.sync import sync_to_async

from assistant.bot.services.context_service.steps.base import ContextProcessingStep, ai_debugger
from assistant.bot.services.context_service.utils import add_system_message
from assistant.bot.services.schema_service import json_prompt
from assistant.utils.fuzzy import extract_bests
from assistant.utils.repeat_until import repeat_until

MIN_TITLE_SCORE = 90


class ChooseDocsStep(ContextProcessingStep):
    debug_info_key = "choice"

    @ai_debugger
    async def run(self):
        documents = list(self._state.documents or [])[:10]
        if not documents:
            return
        titles = await sync_to_async(lambda: [d.wiki.path.replace(" / ", ". ") for d in documents])()
        choices = "\n".join(dict.fromkeys(f"- {t}" for t in titles))
        messages = add_system_message(self._state.messages, (
            f"You can answer the user using information from these documents:\n{choices}\n"
            "However, you must choose up to 3 documents from the list above to get details.\n"
            f"Give the rows from the list above that relate to the user's question:\n```\n"
            f"{self._state.user_question}\n```\n"
            "Give each selected row in full - EXACTLY as it represented in the list.\n"
            "Do not hesitate to provide MULTIPLE rows if necessary.\n"
            "If none of the documents are relevant to the user's question, just provide an empty list.\n"
            f"{json_prompt(['choose_documents'])}"))
        chosen: List = []

        def check(resp) -> bool:
            nonlocal chosen
            if not isinstance(resp.result, dict) or "documents" not in resp.result:
                return False
            picked = [self._select_doc(documents, titles, t) for t in resp.result["documents"] or []]
            if any(d is None for d in picked) or len({d.id for d in picked}) != len(picked):
                return False
            chosen = picked
            return True

        await repeat_until(self._fast_ai.get_response, messages, max_tokens=256, json_format=True, condition=check)
        self._debug_info["chosen"] = [f"[{d.id}] {d.name}" for d in chosen]
        merged = list(self._state.documents[:2]) + chosen
        self._state.documents = list({d.id: d for d in merged}.values())

    @staticmethod
    def _select_doc(documents, titles, title) -> Optional[object]:
        by_title = dict(zip(titles, documents))
        best = extract_bests(str(title).lstrip("- "), list(by_title), limit=1)
        if not best or best[0][1] < MIN_TITLE_SCORE:
            return None
        return by_title[best[0][0]]
