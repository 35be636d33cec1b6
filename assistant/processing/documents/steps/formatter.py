"""LLM re-formatting of a section to Markdown (reference documents/steps/formatter.py:10-39).
Unlike the reference (which only changed the in-memory object) the formatted text is saved."""
from assistant.processing.documents.steps.base import DocumentProcessingStep
from assistant.processing.utils import expected_language, json_prompt, language_ok
from assistant.utils.repeat_until import repeat_until


class DocumentFormatStep(DocumentProcessingStep):
    ai_model_setting = "FORMAT_DOCUMENTS_AI_MODEL"

    @staticmethod
    def prompt(name: str, content: str) -> str:
        return (f"Below is the raw text of a document titled \"{name}\":\n```\n{content}\n```\n\n"
                "Rewrite it in the most readable form using Markdown. Do not drop any information, keep the "
                "meaning exactly and keep the original language.\n"
                f"{json_prompt('format_document')}")

    async def run(self):
        content = (self._document.content or "").replace("\t", " " * 4).strip()
        if not content:
            return
        lang = expected_language(content)
        resp = await repeat_until(
            self._ai.prompt, self.prompt(self._document.name, content), json_format=True,
            condition=lambda r: isinstance(r.result.get("text"), str) and len(r.result["text"]) >= 2
            and language_ok([r.result["text"]], lang))
        self._document.content = resp.result["text"]
        await self._repo.save_document_content(self._document)
