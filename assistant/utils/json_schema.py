"""JSON example schemas embedded into prompts (reference utils/json_schema.py:19-32)."""
from __future__ import annotations

import os


class JSONSchema:
    def __init__(self, schemas_dir: str):
        self._schemas_dir = schemas_dir

    def get_schema(self, name: str) -> str:
        with open(os.path.join(self._schemas_dir, f"{name}.json"), encoding="utf-8") as f:
            body = f.read().strip()
        return f"```json\n{body}\n```\n"

    def get_prompt(self, schema, do_escape: bool = False) -> str:
        if isinstance(schema, (list, tuple)):
            head = "Answer with a JSON response that strictly matches one of the following examples:\n"
            body = "".join(self.get_schema(s) for s in schema)
        else:
            head = "Answer with a JSON response that strictly matches the following example:\n"
            body = self.get_schema(schema)
        tail = "Do not forget to escape special characters in the JSON like \\n.\n" if do_escape else ""
        return head + body + tail
