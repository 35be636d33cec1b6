"""Dialog persistence helpers (reference bot/services/dialog_service.py:17-138)."""
from __future__ import annotations

import base64
import io
import logging
from datetime import timedelta
from typing import List, Optional

from django.core.files.base import ContentFile
from django.utils import timezone

from assistant.ai.domain import Message as GPTMessage
from assistant.ai.services.ai_service import calculate_ai_cost
from assistant.bot.domain import Photo, SingleAnswer
from assistant.bot.models import Dialog, Instance, Message, Role

logger = logging.getLogger(__name__)


def get_gpt_messages(dialog: Dialog, system_text: str, last_message_id: int = None) -> List[GPTMessage]:
    """System prompt + every stored message of the dialog; ``/continue`` becomes a system turn, photos
    become base64 ``images``.  History is not truncated (as in the reference)."""
    messages: List[GPTMessage] = [{"role": "system", "content": system_text}] if system_text else []
    for m in dialog.messages.select_related("role").order_by("timestamp", "id"):
        if last_message_id and m.id > last_message_id:
            continue
        if m.text == "/continue":
            messages.append({"role": "system", "content": "Continue"})
            continue
        images = None
        if m.photo:
            with m.photo.open("rb") as f:
                images = [base64.b64encode(f.read()).decode("ascii")]
        messages.append({"role": m.role.name, "content": m.text, "images": images})
    return messages


def get_dialog(instance: Instance, ttl: timedelta = None) -> Dialog:
    """The instance's open dialog if its last message is newer than ``ttl``; otherwise close it and
    start a new one."""
    last = (Message.objects.filter(dialog__instance=instance, dialog__is_completed=False)
            .select_related("dialog").order_by("-timestamp").first())
    if last and (ttl is None or last.timestamp > timezone.now() - ttl):
        return last.dialog
    if last:
        Dialog.objects.filter(pk=last.dialog_id).update(is_completed=True)
    return Dialog.objects.create(instance=instance)


def get_last_message(dialog: Dialog) -> Optional[Message]:
    return Message.objects.filter(dialog=dialog).order_by("-timestamp").first()


def create_user_message(dialog: Dialog, message_id: int, text: str = None, photo: Photo = None,
                        phone_number: str = None) -> Message:
    role, _ = Role.objects.get_or_create(name="user")
    photo_file = None
    if photo:
        photo_file = ContentFile(io.BytesIO(photo.content).getvalue(), name=f"{photo.file_id}.{photo.extension}")
    if phone_number:
        text = f"{text}\nPhone number: {phone_number}" if text else f"Phone number: {phone_number}"
    m, _ = Message.objects.get_or_create(dialog=dialog, message_id=message_id, role=role,
                                         defaults={"text": text, "photo": photo_file})
    return m


def create_bot_message(dialog: Dialog, answer: SingleAnswer) -> Message:
    role, _ = Role.objects.get_or_create(name="assistant")
    m, _ = Message.objects.get_or_create(dialog=dialog, role=role, text=answer.raw_text, cost_details=answer.usage,
                                         cost=sum(calculate_ai_cost(u) for u in answer.usage))
    return m


def have_existing_answers(user_message: Message) -> bool:
    return Message.objects.filter(dialog=user_message.dialog, role__name="assistant",
                                  id__gt=user_message.id).exists()
