"""Document processors (reference documents/processor.py:21-73).

``DefaultDocumentProcessor``: Format -> ExtractSentences -> GenerateQuestions -> SentencesEmbeddings ->
QuestionsEmbeddings -> MergeQuestions.  ``settings.DOCUMENT_PROCESSOR_CLASSES`` maps a bot codename to a
processor class path; the default path is importable (the reference's lacked the ``assistant.`` prefix).
"""
from __future__ import annotations

import logging
from abc import ABC, abstractmethod
from functools import lru_cache
from typing import List, Type

from assistant.bot.utils import import_string
from assistant.conf import settings
from assistant.processing.documents.steps.base import DocumentProcessingStep
from assistant.processing.documents.steps.embeddings import QuestionsEmbeddingsStep, SentencesEmbeddingsStep
from assistant.processing.documents.steps.formatter import DocumentFormatStep
from assistant.processing.documents.steps.questions import GenerateQuestionsStep, MergeQuestionsStep
from assistant.processing.documents.steps.sentences import ExtractSentencesStep

logger = logging.getLogger(__name__)

DEFAULT_PROCESSOR = "assistant.processing.documents.processor.DefaultDocumentProcessor"


class DocumentProcessor(ABC):
    @property
    @abstractmethod
    def steps(self) -> List[Type[DocumentProcessingStep]]: ...

    async def process(self, document, repository):
        for step_cls in self.steps:
            logger.info("step %s on document %s", step_cls.__name__, getattr(document, "id", None))
            await step_cls(document, repository).run()


class DefaultDocumentProcessor(DocumentProcessor):
    @property
    def steps(self):
        return [DocumentFormatStep, ExtractSentencesStep, GenerateQuestionsStep, SentencesEmbeddingsStep,
                QuestionsEmbeddingsStep, MergeQuestionsStep]


@lru_cache
def get_document_processor(bot_codename: str) -> DocumentProcessor:
    path = (settings.get("DOCUMENT_PROCESSOR_CLASSES") or {}).get(bot_codename, DEFAULT_PROCESSOR)
    logger.info("document processor %s for bot %s", path, bot_codename)
    return import_string(path)()


async def process_document(document, repository, bot_codename: str = None):
    if bot_codename is None:
        from assistant.utils.sync import sync_to_async
        bot_codename = await sync_to_async(
            lambda: document.wiki.bot.codename if getattr(document.wiki, "bot_id", None) else "default")()
    await get_document_processor(bot_codename).process(document, repository)
