from typing import List

from assistant.ai.domain import Message


def add_system_message(messages: List[Message], content: str) -> List[Message]:
    """A new list with a trailing system message (the input list is not modified)."""
    return list(messages) + [Message(role="system", content=content)]


def get_list_str(items: List[str]) -> str:
    return "\n".join(f"- {s}" for s in items)


def get_numerical_list_str(items: List[str]) -> str:
    return "\n".join(f"{i + 1}. `{s}`" for i, s in enumerate(items))
