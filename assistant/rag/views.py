"""RAG query endpoint (the README of the reference advertised ``/api/rag/query/`` but never shipped it).

POST /api/v1/rag/query/ {"bot": codename, "question": str, "history": [{role, content}]?, "max_tokens"?}
-> {"answer": str, "documents": [{id, name, path}], "debug": {...}}: one pass of the bot's context
pipeline (classification, retrieval, FillInfo, FinalPrompt) and the strong model, without a dialog."""
import asyncio
import time

from rest_framework import permissions, serializers
from rest_framework.response import Response
from rest_framework.views import APIView

from assistant.bot.chat_completion import ChatCompletion
from assistant.bot.models import Bot
from assistant.bot.resource_manager import ResourceManager
from assistant.conf import settings


class TurnSerializer(serializers.Serializer):
    role = serializers.ChoiceField(choices=["user", "assistant", "system"])
    content = serializers.CharField(allow_blank=True)


class RAGQuerySerializer(serializers.Serializer):
    bot = serializers.SlugRelatedField("codename", queryset=Bot.objects.all())
    question = serializers.CharField()
    history = TurnSerializer(many=True, required=False)
    max_tokens = serializers.IntegerField(required=False, min_value=1, max_value=8192)


class RAGQueryView(APIView):
    permission_classes = [permissions.IsAuthenticated]

    def post(self, request):
        req = RAGQuerySerializer(data=request.data)
        req.is_valid(raise_exception=True)
        bot = req.validated_data["bot"]
        messages = [{"role": "system", "content": bot.system_text}] if bot.system_text else []
        messages += [dict(m) for m in req.validated_data.get("history", [])]
        messages.append({"role": "user", "content": req.validated_data["question"]})
        completion = ChatCompletion(
            bot=bot, resource_manager=ResourceManager(bot.codename, settings.get("BOT_DEFAULT_LANGUAGE", "ru")),
            fast_ai_model=settings.get("DIALOG_FAST_AI_MODEL") or settings.DEFAULT_AI_MODEL,
            strong_ai_model=settings.get("DIALOG_STRONG_AI_MODEL") or settings.DEFAULT_AI_MODEL)
        debug = {}
        t0 = time.time()
        resp = asyncio.run(completion.generate_answer(messages, debug_info=debug,
                                                      max_tokens=req.validated_data.get("max_tokens", 1024)))
        debug["total"] = {"took": time.time() - t0}
        docs = debug.get("embedding_search", {}).get("documents", [])
        return Response({"answer": resp.result if isinstance(resp.result, str) else str(resp.result),
                         "documents": docs, "usage": resp.usage or {}, "debug": debug})
