"""Telegram platform over the raw Bot API (reference bot/platforms/telegram/platform.py).

The reference depends on python-telegram-bot; this implementation speaks the HTTP Bot API directly
(aiohttp when available, urllib in a worker thread otherwise), so it has no extra dependency and the
transport can be swapped in tests.  Behaviour kept from the reference:

  * updates: message (text / caption, largest photo downloaded, contact phone) and callback_query
    (text = callback data, chat = the pressing user); anything else raises ``UnknownUpdate``
  * inline keyboard for ``answer.buttons``; reply keyboard for ``answer.reply_keyboard`` (one-time when
    it requests contact/location); otherwise the reply keyboard is removed
  * audio is sent before text; text goes as MarkdownV2 and falls back to plain text on a parse error
  * 403 Forbidden -> ``UserUnavailableError`` unless the reason is a kicked bot, deleted group or
    deactivated user (those are logged and dropped)
"""
from __future__ import annotations

import asyncio
import json
import logging
import urllib.error
import urllib.request
import uuid
from typing import Any, Callable, Dict, Optional

from assistant.bot.domain import BotPlatform, Photo, SingleAnswer, UnknownUpdate, Update, User
from assistant.bot.exceptions import UserUnavailableError
from assistant.bot.platforms.telegram.format import TelegramMarkdownV2FormattedText

logger = logging.getLogger(__name__)

API_ROOT = "https://api.telegram.org"
_SILENT_FORBIDDEN = ("bot was kicked", "group chat was deleted", "user is deactivated")


class TelegramError(Exception):
    def __init__(self, message: str, status: int = 0, method: str = ""):
        super().__init__(message)
        self.message = message
        self.status = status
        self.method = method


class BadRequest(TelegramError):
    pass


class Forbidden(TelegramError):
    pass


def _raise_for(method: str, status: int, payload: Dict) -> Any:
    if payload.get("ok"):
        return payload.get("result")
    desc = payload.get("description") or f"HTTP {status}"
    code = payload.get("error_code", status)
    if code == 403:
        raise Forbidden(desc, code, method)
    if code == 400:
        raise BadRequest(desc, code, method)
    raise TelegramError(desc, code, method)


class TelegramAPI:
    """Minimal async Bot API client.  ``transport(method, params, files) -> (status, json)`` can be
    injected (tests); by default it posts JSON (or multipart when files are attached)."""

    def __init__(self, token: str, transport: Optional[Callable] = None, api_root: str = API_ROOT,
                 timeout: float = 30.0):
        self.token = token
        self.api_root = api_root.rstrip("/")
        self.timeout = timeout
        self._transport = transport

    async def call(self, method: str, files: Optional[Dict[str, tuple]] = None, **params) -> Any:
        params = {k: v for k, v in params.items() if v is not None}
        if self._transport is not None:
            status, payload = await self._transport(method, params, files)
        else:
            status, payload = await self._http(method, params, files)
        return _raise_for(method, status, payload)

    async def download(self, file_path: str) -> bytes:
        url = f"{self.api_root}/file/bot{self.token}/{file_path}"
        if self._transport is not None:
            status, payload = await self._transport("__download__", {"file_path": file_path}, None)
            return payload
        return await asyncio.to_thread(lambda: urllib.request.urlopen(url, timeout=self.timeout).read())

    async def _http(self, method: str, params: Dict, files: Optional[Dict[str, tuple]]):
        url = f"{self.api_root}/bot{self.token}/{method}"
        try:
            import aiohttp
        except ImportError:  # pragma: no cover - aiohttp is in the image
            aiohttp = None
        if aiohttp is not None:
            timeout = aiohttp.ClientTimeout(total=self.timeout)
            async with aiohttp.ClientSession(timeout=timeout) as session:
                if files:
                    form = aiohttp.FormData()
                    for k, v in params.items():
                        form.add_field(k, v if isinstance(v, str) else json.dumps(v))
                    for field, (filename, content) in files.items():
                        form.add_field(field, content, filename=filename or field)
                    resp = await session.post(url, data=form)
                else:
                    resp = await session.post(url, json=params)
                async with resp:
                    return resp.status, await resp.json(content_type=None)
        return await asyncio.to_thread(self._urllib_post, url, params, files)

    def _urllib_post(self, url: str, params: Dict, files):
        if files:
            boundary = uuid.uuid4().hex
            chunks = []
            for k, v in params.items():
                v = v if isinstance(v, str) else json.dumps(v)
                chunks.append(f'--{boundary}\r\nContent-Disposition: form-data; name="{k}"\r\n\r\n{v}\r\n'.encode())
            for field, (filename, content) in files.items():
                chunks.append(f'--{boundary}\r\nContent-Disposition: form-data; name="{field}"; '
                              f'filename="{filename or field}"\r\n\r\n'.encode() + bytes(content) + b"\r\n")
            chunks.append(f"--{boundary}--\r\n".encode())
            body, ctype = b"".join(chunks), f"multipart/form-data; boundary={boundary}"
        else:
            body, ctype = json.dumps(params).encode(), "application/json"
        req = urllib.request.Request(url, data=body, headers={"Content-Type": ctype})
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                return r.status, json.loads(r.read())
        except urllib.error.HTTPError as e:
            try:
                return e.code, json.loads(e.read())
            except ValueError:
                return e.code, {"ok": False, "error_code": e.code, "description": str(e)}


def _reply_markup(answer: SingleAnswer) -> Dict:
    if answer.buttons:
        return {"inline_keyboard": [[{k: v for k, v in {"text": b.text, "callback_data": b.callback_data,
                                                        "url": b.url}.items() if v is not None}
                                     for b in row] for row in answer.buttons]}
    if answer.reply_keyboard:
        flat = [b for row in answer.reply_keyboard for b in row]
        contact = any(getattr(b, "request_contact", False) for b in flat)
        location = any(getattr(b, "request_location", False) for b in flat)
        rows = []
        for row in answer.reply_keyboard:
            out_row = []
            for b in row:
                btn = {"text": getattr(b, "text", b)}
                if contact:
                    btn["request_contact"] = True
                if location:
                    btn["request_location"] = True
                out_row.append(btn)
            rows.append(out_row)
        return {"keyboard": rows, "one_time_keyboard": contact or location, "resize_keyboard": True}
    return {"remove_keyboard": True}


class TelegramBotPlatform(BotPlatform):
    def __init__(self, token: str, api: Optional[TelegramAPI] = None):
        self.api = api or TelegramAPI(token)

    @property
    def codename(self) -> str:
        return "telegram"

    async def convert_telegram_update(self, data: Dict) -> Update:
        message = data.get("message")
        callback = data.get("callback_query")
        src = (message or {}).get("from") or (callback or {}).get("from")
        user = User(id=str(src["id"]), username=src.get("username"), first_name=src.get("first_name"),
                    last_name=src.get("last_name"), language_code=src.get("language_code")) if src else None
        photo = phone = None
        if message:
            chat_id = message["chat"]["id"]
            message_id = message.get("message_id")
            text = message.get("text")
            if message.get("contact"):
                phone = message["contact"].get("phone_number")
            if message.get("photo"):
                largest = message["photo"][-1]
                info = await self.api.call("getFile", file_id=largest["file_id"])
                content = await self.api.download(info["file_path"])
                photo = Photo(file_id=largest.get("file_unique_id", largest["file_id"]),
                              extension=info["file_path"].rsplit(".", 1)[-1], content=bytes(content))
                text = text or message.get("caption")
        elif callback:
            chat_id = callback["from"]["id"]
            message_id = (callback.get("message") or {}).get("message_id")
            text = callback.get("data")
        else:
            raise UnknownUpdate("Unknown update type")
        return Update(chat_id=str(chat_id), message_id=message_id, text=text, photo=photo, user=user,
                      phone_number=phone)

    async def get_update(self, request) -> Update:
        data = getattr(request, "data", request)
        if isinstance(data, (bytes, str)):
            data = json.loads(data)
        logger.debug("Got Telegram request: %s", data)
        return await self.convert_telegram_update(data)

    @staticmethod
    def _handle_forbidden(chat_id: str, e: Forbidden) -> None:
        reason = e.message.lower()
        if any(s in reason for s in _SILENT_FORBIDDEN):
            logger.warning("Delivery to %s forbidden (%s); dropping", chat_id, e.message)
            return
        raise UserUnavailableError(chat_id) from e

    async def post_answer(self, chat_id: str, answer: SingleAnswer):
        markup = _reply_markup(answer)
        text = TelegramMarkdownV2FormattedText(answer.text) if answer.text else None
        sent = False
        if answer.audio:
            try:
                await self.api.call("sendAudio", chat_id=chat_id,
                                    reply_markup=None if text else markup,
                                    files={"audio": (answer.audio.filename or "audio.mp3", answer.audio.content)})
                sent = True
            except Forbidden as e:
                self._handle_forbidden(chat_id, e)
                return
            except BadRequest as e:
                logger.error("Failed to send audio to %s: %s", chat_id, e)
        if text:
            attempts = ((str(text), "MarkdownV2"), (text.raw_text, None))
            for body, mode in attempts:
                try:
                    await self.api.call("sendMessage", chat_id=chat_id, text=body, parse_mode=mode,
                                        reply_markup=markup,
                                        disable_web_page_preview=answer.disable_web_page_preview)
                    sent = True
                    break
                except BadRequest as e:
                    if mode and "can't parse" in e.message.lower():
                        logger.warning("MarkdownV2 rejected (%s); resending as plain text", e.message)
                        continue
                    logger.error("Failed to send message to %s: %s", chat_id, e)
                    break
                except Forbidden as e:
                    self._handle_forbidden(chat_id, e)
                    return
        if not sent:
            logger.warning("Nothing delivered to %s", chat_id)

    async def action_typing(self, chat_id):
        await self.api.call("sendChatAction", chat_id=chat_id, action="typing")

    async def set_webhook(self, url: str, secret_token: Optional[str] = None):
        return await self.api.call("setWebhook", url=url, secret_token=secret_token)

    async def get_updates(self, offset: Optional[int] = None, timeout: int = 30):
        return await self.api.call("getUpdates", offset=offset, timeout=timeout)
