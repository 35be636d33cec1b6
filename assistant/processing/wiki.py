"""Wiki page -> sections (reference processing/wiki.py:16-99).

Pages shorter than ``DOCUMENT_MAX_LENGTH`` characters become one section named after the title.  Longer
pages: one LLM call proposes >= 2 section titles, then one call per section returns its text word for
word.  Each section is stored as a ``Document`` of a new ``WikiDocumentProcessing`` run."""
from __future__ import annotations

import logging
from typing import List

from assistant.ai.dialog import AIDialog
from assistant.processing.documents.steps.base import model_setting
from assistant.processing.utils import expected_language, json_prompt, language_ok
from assistant.conf import settings
from assistant.utils.repeat_until import repeat_until

logger = logging.getLogger(__name__)


class WikiDocumentSplitter:
    def __init__(self, wiki, repository):
        self._wiki = wiki
        self._repo = repository
        self._ai = AIDialog(model_setting("SPLIT_DOCUMENTS_AI_MODEL"))
        self._lang = expected_language(wiki.content or "")

    async def run(self):
        processing = await self._repo.start_processing(self._wiki)
        names = await self.section_names()
        logger.info("wiki %s: sections %s", getattr(self._wiki, "id", None), names)
        for name in names:
            text = await self.section_text(names, name)
            await self._repo.add_document(processing, self._wiki, name, text)
        return processing

    def _page(self) -> str:
        return (f"Here is a long document titled \"{self._wiki.title}\":\n"
                f"```\n{self._wiki.content.strip()}\n```\n\n")

    async def section_names(self) -> List[str]:
        content = self._wiki.content or ""
        if not content:
            return []
        if len(content) < int(settings.get("DOCUMENT_MAX_LENGTH", 1000)):
            return [self._wiki.title]
        prompt = (self._page() + "Split it into two or more parts along its meaning, choosing the number of parts "
                  "that fits best, and propose a title for each part in the document's language.\n"
                  f"{json_prompt('split_document_get_names')}")
        resp = await repeat_until(
            self._ai.prompt, prompt, json_format=True,
            condition=lambda r: isinstance(r.result.get("names"), list) and len(r.result["names"]) >= 2
            and all(isinstance(n, str) for n in r.result["names"]) and language_ok(r.result["names"], self._lang))
        return resp.result["names"]

    async def section_text(self, names: List[str], name: str) -> str:
        if len(names) == 1 and name == names[0]:
            return self._wiki.content
        listing = "\n- ".join(names)
        prompt = (self._page() + f"The document is divided into {len(names)} parts:\n- {listing}\n"
                  f"Return the text of the part \"{name}\", matching the original word for word, in the original "
                  "language.\n"
                  f"{json_prompt('split_document_get_section', do_escape=True)}")
        resp = await repeat_until(
            self._ai.prompt, prompt, json_format=True,
            condition=lambda r: isinstance(r.result.get("text"), str) and language_ok([r.result["text"]], self._lang))
        return resp.result["text"]


async def split_wiki_document(wiki, repository):
    return await WikiDocumentSplitter(wiki, repository).run()


async def ingest_wiki(wiki, repository, bot_codename: str = "default"):
    """Whole pipeline in-process: split, process every section, finalize (the Celery tasks run the
    same three phases as a fan-out / fan-in chain)."""
    from assistant.processing.documents.processor import process_document

    processing = await split_wiki_document(wiki, repository)
    docs = [d for d in getattr(repository, "documents", {}).values() if d.processing is processing] \
        if hasattr(repository, "documents") else None
    if docs is None:
        from assistant.utils.sync import sync_to_async
        docs = await sync_to_async(lambda: list(processing.documents.all()))()
    for d in docs:
        await process_document(d, repository, bot_codename)
    await repository.finalize(processing)
    return processing
