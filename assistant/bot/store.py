"""Persistence seam of the conversation layer.

The reference's ``AssistantBot`` talks to the Django ORM directly (reference bot/assistant_bot.py:
53-517 via ``sync_to_async`` everywhere).  Here the bot depends on a small async ``BotStore``:
``DjangoBotStore`` is the production implementation (ORM, used by the Celery task, the REST API and
the management commands); ``MemoryBotStore`` keeps the same records in process memory, which makes
the whole update -> answer flow runnable and testable without a database (and is what the console
``chat`` command can use with ``--memory``).

Records expose the attribute names of the ORM models (``instance.state``, ``bot.codename``,
``message.message_id`` ...), so bot code is identical for both stores.
"""
from __future__ import annotations

import dataclasses
import itertools
import threading
import time
import uuid
from abc import ABC, abstractmethod
from typing import Any, Dict, List, Optional

from assistant.ai.domain import Message as GPTMessage
from assistant.bot.domain import Photo, SingleAnswer
from assistant.rag.knowledge import EmptyKnowledgeBase
from assistant.utils.sync import sync_to_async


class BotStore(ABC):
    @abstractmethod
    async def save_instance(self, instance, fields: List[str]) -> None: ...

    @abstractmethod
    async def save_dialog(self, dialog, fields: List[str]) -> None: ...

    @abstractmethod
    async def gpt_messages(self, dialog, system_text: Optional[str]) -> List[GPTMessage]: ...

    @abstractmethod
    async def last_user_message(self, dialog): ...

    @abstractmethod
    async def has_answers_after(self, user_message) -> bool: ...

    @abstractmethod
    async def has_messages_after(self, dialog, message_id: int) -> bool: ...

    @abstractmethod
    async def add_user_message(self, dialog, message_id: int, text: str = None, photo: Photo = None,
                               phone_number: str = None): ...

    @abstractmethod
    async def add_bot_message(self, dialog, answer: SingleAnswer): ...

    @abstractmethod
    async def complete_dialogs(self, instance) -> int: ...

    async def get_document(self, bot, doc_id) -> Optional[Any]:
        return None

    async def get_wiki(self, bot, wiki_id) -> Optional[Any]:
        return None


# --------------------------------------------------------------------------------- in-memory store

@dataclasses.dataclass
class BotRecord:
    codename: str
    system_text: Optional[str] = None
    start_text: Optional[str] = None
    help_text: Optional[str] = None
    is_whitelist_enabled: bool = False
    telegram_whitelist: str = ""
    telegram_token: Optional[str] = None
    username: Optional[str] = None
    id: int = 1
    knowledge: Any = dataclasses.field(default_factory=lambda: EmptyKnowledgeBase())


@dataclasses.dataclass
class BotUserRecord:
    user_id: str
    platform: str = "console"
    username: Optional[str] = None
    language: Optional[str] = None
    phone_number: Optional[str] = None
    id: int = 1


@dataclasses.dataclass
class InstanceRecord:
    bot: BotRecord
    user: BotUserRecord
    state: Dict = dataclasses.field(default_factory=dict)
    is_unavailable: bool = False
    id: int = 1


@dataclasses.dataclass
class DialogRecord:
    instance: InstanceRecord
    is_completed: bool = False
    state: Dict = dataclasses.field(default_factory=dict)
    id: str = dataclasses.field(default_factory=lambda: str(uuid.uuid4()))


@dataclasses.dataclass
class MessageRecord:
    dialog: DialogRecord
    role: str
    text: Optional[str]
    message_id: Optional[int] = None
    photo: Optional[Photo] = None
    cost_details: Any = None
    timestamp: float = dataclasses.field(default_factory=time.time)
    id: int = 0


class MemoryBotStore(BotStore):
    def __init__(self):
        self._messages: List[MessageRecord] = []
        self._dialogs: List[DialogRecord] = []
        self._ids = itertools.count(1)
        self._lock = threading.Lock()
        self.documents: Dict[Any, Any] = {}
        self.wikis: Dict[Any, Any] = {}

    # record helpers ---------------------------------------------------------------------------
    def open_dialog(self, instance: InstanceRecord) -> DialogRecord:
        with self._lock:
            for d in reversed(self._dialogs):
                if d.instance is instance and not d.is_completed:
                    return d
            d = DialogRecord(instance=instance)
            self._dialogs.append(d)
            return d

    def messages(self, dialog) -> List[MessageRecord]:
        return [m for m in self._messages if m.dialog is dialog]

    # BotStore ---------------------------------------------------------------------------------
    async def save_instance(self, instance, fields):
        return None

    async def save_dialog(self, dialog, fields):
        return None

    async def gpt_messages(self, dialog, system_text):
        out: List[GPTMessage] = [{"role": "system", "content": system_text}] if system_text else []
        for m in self.messages(dialog):
            if m.text == "/continue":
                out.append({"role": "system", "content": "Continue"})
            else:
                out.append({"role": m.role, "content": m.text})
        return out

    async def last_user_message(self, dialog):
        users = [m for m in self.messages(dialog) if m.role == "user"]
        return users[-1] if users else None

    async def has_answers_after(self, user_message):
        return any(m.role == "assistant" and m.id > user_message.id for m in self.messages(user_message.dialog))

    async def has_messages_after(self, dialog, message_id):
        return any(m.message_id is not None and message_id is not None and m.message_id > message_id
                   for m in self.messages(dialog))

    async def add_user_message(self, dialog, message_id, text=None, photo=None, phone_number=None):
        if phone_number:
            text = f"{text}\nPhone number: {phone_number}" if text else f"Phone number: {phone_number}"
        with self._lock:
            for m in self._messages:
                if m.dialog is dialog and m.message_id == message_id and m.role == "user":
                    return m
            m = MessageRecord(dialog=dialog, role="user", text=text, message_id=message_id, photo=photo,
                              id=next(self._ids))
            self._messages.append(m)
            return m

    async def add_bot_message(self, dialog, answer):
        with self._lock:
            m = MessageRecord(dialog=dialog, role="assistant", text=answer.raw_text, cost_details=answer.usage,
                              id=next(self._ids))
            self._messages.append(m)
            return m

    async def complete_dialogs(self, instance):
        n = 0
        for d in self._dialogs:
            if d.instance is instance and not d.is_completed:
                d.is_completed, n = True, n + 1
        return n

    async def get_document(self, bot, doc_id):
        return self.documents.get(str(doc_id))

    async def get_wiki(self, bot, wiki_id):
        return self.wikis.get(str(wiki_id))


# ------------------------------------------------------------------------------------ Django store

class DjangoBotStore(BotStore):
    """ORM-backed store (reference bot/services/dialog_service.py semantics)."""

    async def save_instance(self, instance, fields):
        await sync_to_async(instance.save)(update_fields=fields)

    async def save_dialog(self, dialog, fields):
        await sync_to_async(dialog.save)(update_fields=fields)

    async def gpt_messages(self, dialog, system_text):
        from assistant.bot.services.dialog_service import get_gpt_messages
        return await sync_to_async(get_gpt_messages)(dialog, system_text)

    async def last_user_message(self, dialog):
        from assistant.bot.models import Message
        return await sync_to_async(
            lambda: Message.objects.filter(dialog_id=dialog.id, role__name="user").order_by("timestamp", "id").last())()

    async def has_answers_after(self, user_message):
        from assistant.bot.services.dialog_service import have_existing_answers
        return await sync_to_async(have_existing_answers)(user_message)

    async def has_messages_after(self, dialog, message_id):
        return await sync_to_async(dialog.messages.filter(message_id__gt=message_id).exists)()

    async def add_user_message(self, dialog, message_id, text=None, photo=None, phone_number=None):
        from assistant.bot.services.dialog_service import create_user_message
        return await sync_to_async(create_user_message)(dialog, message_id, text, photo, phone_number)

    async def add_bot_message(self, dialog, answer):
        from assistant.bot.services.dialog_service import create_bot_message
        return await sync_to_async(create_bot_message)(dialog, answer)

    async def complete_dialogs(self, instance):
        from assistant.bot.models import Dialog
        return await sync_to_async(
            lambda: Dialog.objects.filter(instance=instance, is_completed=False).update(is_completed=True))()

    async def get_document(self, bot, doc_id):
        from assistant.storage.models import Document

        def get():
            return Document.objects.filter(wiki__bot=bot, id=doc_id).select_related("wiki").first()
        return await sync_to_async(get)()

    async def get_wiki(self, bot, wiki_id):
        from assistant.storage.models import WikiDocument
        return await sync_to_async(lambda: WikiDocument.objects.filter(bot=bot, id=wiki_id).first())()
