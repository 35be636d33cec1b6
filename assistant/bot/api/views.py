"""Conversation REST API (reference bot/api/views.py:19-223).

  /bots/                          read-only bot list (lookup by codename)
  /bots/<codename>/chat/completions  OpenAI-style completion through the bot's context pipeline
                                  (present but disabled in the reference; enabled here)
  /dialogs/                       CRUD
  /dialogs/<id>/messages/         list / retrieve / create; create runs the bot synchronously under
                                  the instance lock and returns the user message with its answers
"""
import asyncio
import logging
import time

from django.shortcuts import get_object_or_404
from rest_framework import mixins, permissions, status, viewsets
from rest_framework.decorators import action
from rest_framework.response import Response

from assistant.bot.api.serializers import (AnsweredMessageSerializer, BotSerializer, ChatCompletionRequestSerializer,
                                           DialogSerializer, MessageSerializer)
from assistant.bot.domain import Update
from assistant.bot.models import Bot, Dialog, Message
from assistant.bot.platforms.api import CollectingPlatform
from assistant.bot.resource_manager import ResourceManager
from assistant.bot.services.dialog_service import create_user_message
from assistant.bot.services.instance_service import InstanceLock
from assistant.bot.store import DjangoBotStore
from assistant.bot.utils import get_bot_class
from assistant.conf import settings
from assistant.utils.sync import async_to_sync

logger = logging.getLogger(__name__)


class BotViewSet(viewsets.ReadOnlyModelViewSet):
    queryset = Bot.objects.order_by("id")
    serializer_class = BotSerializer
    lookup_field = "codename"

    @action(detail=True, methods=["post"], url_path="chat/completions",
            permission_classes=[permissions.IsAuthenticated])
    def chat_completion(self, request, codename=None):
        from assistant.bot.chat_completion import ChatCompletion

        req = ChatCompletionRequestSerializer(data=request.data)
        req.is_valid(raise_exception=True)
        bot = self.get_object()
        t0 = time.time()
        completion = ChatCompletion(
            bot=bot, resource_manager=ResourceManager(bot.codename, language=settings.get("BOT_DEFAULT_LANGUAGE", "ru")),
            fast_ai_model=settings.get("DIALOG_FAST_AI_MODEL") or settings.DEFAULT_AI_MODEL,
            strong_ai_model=settings.get("DIALOG_STRONG_AI_MODEL") or settings.DEFAULT_AI_MODEL)
        debug_info = {}
        messages = [dict(m) for m in req.validated_data["messages"]]
        if bot.system_text and messages[0]["role"] != "system":
            messages.insert(0, {"role": "system", "content": bot.system_text})
        response = asyncio.run(completion.generate_answer(messages, debug_info,
                                                          max_tokens=req.validated_data.get("max_tokens", 1024)))
        debug_info["total"] = {"took": time.time() - t0}
        text = response.result if isinstance(response.result, str) else str(response.result)
        return Response({"choices": [{"index": 0, "message": {"role": "assistant", "content": text},
                                      "finish_reason": "length" if response.length_limited else "stop"}],
                         "usage": response.usage or {}}, status=status.HTTP_200_OK)


class DialogViewSet(viewsets.ModelViewSet):
    serializer_class = DialogSerializer
    permission_classes = [permissions.IsAuthenticated]
    queryset = Dialog.objects.select_related("instance", "instance__bot", "instance__user").order_by("created_at")


class MessageViewSet(mixins.CreateModelMixin, mixins.ListModelMixin, mixins.RetrieveModelMixin,
                     viewsets.GenericViewSet):
    serializer_class = MessageSerializer
    permission_classes = [permissions.IsAuthenticated]

    def get_queryset(self):
        dialog = get_object_or_404(Dialog, pk=self.kwargs["dialog_pk"])
        return Message.objects.filter(dialog=dialog).order_by("id")

    def create(self, request, *args, **kwargs):
        dialog = get_object_or_404(Dialog.objects.select_related("instance", "instance__bot", "instance__user"),
                                   pk=self.kwargs["dialog_pk"])
        serializer = self.get_serializer(data=request.data)
        serializer.is_valid(raise_exception=True)
        with InstanceLock(dialog.instance):
            user_message = self._answer(dialog, serializer.validated_data["text"])
        return Response(AnsweredMessageSerializer(user_message).data, status=status.HTTP_201_CREATED,
                        headers=self.get_success_headers(serializer.data))

    def _answer(self, dialog, text):
        message_id = dialog.messages.count()
        create_user_message(dialog, message_id, text)
        user_message = Message.objects.filter(dialog=dialog, role__name="user").order_by("-id").first()
        update = Update(chat_id=str(dialog.id), message_id=message_id, text=text)
        bot = get_bot_class(dialog.instance.bot.codename)(dialog=dialog, platform=CollectingPlatform(),
                                                          store=DjangoBotStore())

        async def run():
            answer = await bot.handle_update(update)
            if answer:
                await bot.on_answer_sent(answer)

        async_to_sync(run)()
        return user_message
