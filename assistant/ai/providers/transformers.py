"""In-process generator on the MI355X engine (replaces the reference's HF ``TransformersProvider``,
ai/providers/transformers.py:9-94).

Same contract: prompt rendered as ``"role: content"`` lines (no chat template; the setting
``ENGINE_CHAT_TEMPLATE`` opts into the checkpoint's own template when it has one), sampling with
top_k=50 / top_p=0.95, JSON mode returns the parsed object (constrained decoding: the text is
one JSON object by construction; the raw string is kept if it still fails to parse), usage reports
prompt/completion token counts, ``length_limited`` when the completion hit the budget.  Differences:
requests from all concurrent callers share one continuous batch on the GPU (``LLMWorker``), and
``max_tokens`` bounds the completion only (the reference's ``max_length`` also counted the prompt).
"""
from __future__ import annotations

import json
import logging
from typing import List

from assistant.ai.domain import AIResponse, Message
from assistant.ai.providers.base import AIProvider

logger = logging.getLogger(__name__)


def render_prompt(messages: List[Message]) -> str:
    return "\n".join(f"{m['role']}: {m['content']}" for m in messages)


class TransformersProvider(AIProvider):
    def __init__(self, model_name: str, local_files_only: bool = True, **engine_kwargs):
        from django_assistant_bot_amd.engine.serving import get_llm_worker

        self._model = model_name
        self._worker = get_llm_worker(model_name, **engine_kwargs)
        self._tokenizer = self._worker.engine.tokenizer

    @property
    def context_size(self) -> int:
        return self._worker.engine.max_model_len

    def calculate_tokens(self, text: str) -> int:
        return self._tokenizer.count_tokens(text)

    async def get_response(self, messages: List[Message], max_tokens: int = 1024,
                           json_format: bool = False, json_schema: dict | None = None) -> AIResponse:
        from django_assistant_bot_amd.engine.llm_engine import SamplingParams

        from assistant.conf import settings

        flag = settings.get("ENGINE_CHAT_TEMPLATE", False)
        flag = flag if isinstance(flag, bool) else str(flag).strip().lower() in ("1", "true", "yes", "on")
        if flag and getattr(self._tokenizer, "has_chat_template", False):
            # the template writes BOS and the role headers itself
            prompt = self._tokenizer.render_chat([{"role": m["role"], "content": m["content"]} for m in messages])
            ids = self._tokenizer.encode(prompt, add_special=False, max_len=self._worker.engine.max_model_len - 1)
        else:
            prompt = render_prompt(messages)
            ids = self._tokenizer.encode(prompt, add_special=True, max_len=self._worker.engine.max_model_len - 1)
        # JSON mode constrains the sampler to one JSON object (engine/json_constraint.py): valid in
        # one generation where the reference retries until json.loads succeeds
        params = SamplingParams(max_new_tokens=max_tokens, temperature=1.0, top_k=50, top_p=0.95,
                                json_mode=bool(json_format), json_schema=json_schema)
        json_format = json_format or json_schema is not None
        out = await self._worker.generate(ids, params)
        text = out.text.strip()
        result = text
        if json_format:
            try:
                result = json.loads(text)
            except json.JSONDecodeError:
                logger.warning("generator returned non-JSON text in JSON mode")
        self._record_attempts(1)
        return AIResponse(result=result,
                          usage={"model": self._model, "prompt_tokens": out.usage["prompt_tokens"],
                                 "completion_tokens": out.usage["completion_tokens"]},
                          length_limited=out.finish_reason == "length")
