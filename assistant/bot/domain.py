"""Platform-independent bot domain: updates, answers, buttons and the platform / bot interfaces
(reference bot/domain.py:14-310).  Pure Python: no Django import (the reference pulled in DRF and
the ORM for type hints only)."""
from __future__ import annotations

import base64
import dataclasses
import logging
from abc import ABC, abstractmethod
from typing import Any, Dict, List, Optional, Union

logger = logging.getLogger(__name__)


class NoMessageFound(Exception):
    pass


class NoResourceFound(Exception):
    pass


class UnknownUpdate(Exception):
    pass


def _b64(data) -> str:
    return base64.b64encode(bytes(data)).decode("ascii")


@dataclasses.dataclass
class User:
    id: str
    username: Optional[str] = None
    first_name: Optional[str] = None
    last_name: Optional[str] = None
    language_code: Optional[str] = None

    def to_dict(self) -> Dict:
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, data: Dict) -> "User":
        return cls(**data)


@dataclasses.dataclass
class CallbackQuery:
    id: str
    from_user: User
    message: Optional[str]
    data: Optional[str]

    def to_dict(self) -> Dict:
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, data: Dict) -> "CallbackQuery":
        d = dict(data)
        d["from_user"] = User.from_dict(d["from_user"]) if isinstance(d["from_user"], dict) else d["from_user"]
        return cls(**d)


@dataclasses.dataclass
class Audio:
    content: bytes
    filename: Optional[str] = None

    def to_dict(self) -> Dict:
        return {"content": _b64(self.content), "filename": self.filename}

    @classmethod
    def from_dict(cls, data: Dict) -> "Audio":
        return cls(content=base64.b64decode(data["content"]), filename=data.get("filename"))


@dataclasses.dataclass
class Photo:
    file_id: str
    extension: str
    content: bytes

    def to_dict(self) -> Dict:
        return {"file_id": self.file_id, "extension": self.extension, "content": _b64(self.content)}

    @classmethod
    def from_dict(cls, data: Dict) -> "Photo":
        return cls(file_id=data["file_id"], extension=data["extension"], content=base64.b64decode(data["content"]))


@dataclasses.dataclass
class Update:
    chat_id: str
    message_id: Optional[int]
    text: Optional[str]
    photo: Optional[Photo] = None
    user: Optional[User] = None
    callback_query: Optional[CallbackQuery] = None
    phone_number: Optional[str] = None

    def to_dict(self) -> Dict:
        return {
            "chat_id": self.chat_id, "message_id": self.message_id, "text": self.text,
            "photo": self.photo.to_dict() if self.photo else None,
            "user": self.user.to_dict() if self.user else None,
            "callback_query": self.callback_query.to_dict() if self.callback_query else None,
            "phone_number": self.phone_number,
        }

    @classmethod
    def from_dict(cls, data: Dict) -> "Update":
        d = dict(data)
        if d.get("user"):
            d["user"] = User.from_dict(d["user"])
        if d.get("photo"):
            d["photo"] = Photo.from_dict(d["photo"])
        if d.get("callback_query"):
            d["callback_query"] = CallbackQuery.from_dict(d["callback_query"])
        return cls(**d)


@dataclasses.dataclass
class Button:
    text: str
    callback_data: Optional[str] = None
    url: Optional[str] = None
    request_contact: Optional[bool] = None
    request_location: Optional[bool] = None

    def to_dict(self) -> Dict:
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, data: Dict) -> "Button":
        return cls(**data)


class SingleAnswer:
    """One outgoing message.  ``raw_text`` falls back to ``text`` (used when storing the dialog)."""

    def __init__(self, text: str = None, thinking: str = None, image_url: str = None, is_markdown: bool = False,
                 reply_keyboard: Any = None, buttons: List[List[Button]] = None, state: Dict = None,
                 raw_text: str = None, usage: List[Dict] = None, debug_info: Dict = None, no_store: bool = False,
                 audio: Optional[Audio] = None, disable_web_page_preview: Optional[bool] = None):
        self.text = text
        self.thinking = thinking
        self.image_url = image_url
        self.is_markdown = is_markdown
        self.reply_keyboard = reply_keyboard
        self.buttons = buttons
        self.state = state
        self.usage = usage or []
        self.debug_info = debug_info or {}
        self.no_store = no_store
        self._raw_text = raw_text
        self.audio = audio
        self.disable_web_page_preview = disable_web_page_preview

    @property
    def raw_text(self):
        return self._raw_text or self.text

    @raw_text.setter
    def raw_text(self, value):
        self._raw_text = value

    @property
    def final_model(self):
        return self.usage[-1].get("model") if self.usage else None

    def to_dict(self) -> Dict:
        return {
            "text": self.text, "thinking": self.thinking, "image_url": self.image_url,
            "is_markdown": self.is_markdown, "reply_keyboard": self.reply_keyboard,
            "buttons": [[b.to_dict() for b in row] for row in self.buttons] if self.buttons else None,
            "state": self.state, "usage": self.usage, "debug_info": self.debug_info, "no_store": self.no_store,
            "raw_text": self._raw_text, "audio": self.audio.to_dict() if self.audio else None,
            "disable_web_page_preview": self.disable_web_page_preview,
        }

    @classmethod
    def from_dict(cls, data: Dict) -> "SingleAnswer":
        d = dict(data)
        if d.get("buttons"):
            d["buttons"] = [[Button.from_dict(b) for b in row] for row in d["buttons"]]
        if d.get("audio"):
            d["audio"] = Audio.from_dict(d["audio"])
        return cls(**d)

    def __repr__(self):
        return f"SingleAnswer(text={self.text!r})"


class MultiPartAnswer:
    """Several messages sent in order; stored only if some part is stored."""

    def __init__(self, parts: List[SingleAnswer] = None, no_store: bool = False, state: Dict = None):
        self.parts = list(parts or [])
        self.state = state or {}
        if no_store:
            self.no_store = True

    def add_part(self, answer: SingleAnswer) -> None:
        self.parts.append(answer)

    def get_parts(self) -> List[SingleAnswer]:
        return self.parts

    @property
    def no_store(self) -> bool:
        return all(p.no_store for p in self.parts)

    @no_store.setter
    def no_store(self, value: bool) -> None:
        for p in self.parts:
            p.no_store = value

    def to_dict(self) -> Dict:
        return {"parts": [p.to_dict() for p in self.parts], "no_store": self.no_store, "state": self.state}

    @classmethod
    def from_dict(cls, data: Dict) -> "MultiPartAnswer":
        d = dict(data)
        parts = [SingleAnswer.from_dict(p) for p in d.pop("parts", [])]
        return cls(parts=parts, **d)


Answer = Union[SingleAnswer, MultiPartAnswer]


def answer_from_dict(data: Dict) -> Answer:
    return MultiPartAnswer.from_dict(data) if "parts" in data else SingleAnswer.from_dict(data)


class BotPlatform(ABC):
    @property
    @abstractmethod
    def codename(self) -> str:
        """Unique platform codename ('telegram', 'console', ...)."""

    @abstractmethod
    async def get_update(self, request) -> Update:
        """Parse an incoming platform request into an ``Update``."""

    @abstractmethod
    async def post_answer(self, chat_id: str, answer: SingleAnswer):
        """Deliver an answer."""

    @abstractmethod
    async def action_typing(self, chat_id):
        """Show the typing indicator."""


class Bot(ABC):
    @abstractmethod
    async def handle_update(self, update: Update) -> Answer:
        pass

    @abstractmethod
    async def on_answer_sent(self, answer: Answer):
        pass
