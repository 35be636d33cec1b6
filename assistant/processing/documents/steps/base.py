"""Document ingest step base (reference processing/documents/steps/base.py)."""
from __future__ import annotations

import logging
from abc import ABC, abstractmethod

from assistant.ai.dialog import AIDialog
from assistant.conf import settings


def model_setting(name: str) -> str:
    """Per-step model (e.g. QUESTIONS_AI_MODEL) falling back to DEFAULT_AI_MODEL."""
    return settings.get(name) or settings.DEFAULT_AI_MODEL


class DocumentProcessingStep(ABC):
    ai_model_setting: str = None

    def __init__(self, document, repository):
        self._document = document
        self._repo = repository
        self._logger = logging.getLogger(self.__class__.__name__)
        self._ai = AIDialog(model_setting(self.ai_model_setting)) if self.ai_model_setting else None

    @abstractmethod
    async def run(self):
        """Process ``self._document`` (mutating it / its rows through the repository)."""
