"""REST serializers of the conversation API (reference bot/api/serializers.py)."""
import uuid

from rest_framework import serializers

from assistant.bot.models import Bot, BotUser, Dialog, Instance, Message


class ChatCompletionMessageSerializer(serializers.Serializer):
    role = serializers.ChoiceField(choices=["system", "user", "assistant"])
    content = serializers.CharField(allow_blank=True)


class ChatCompletionRequestSerializer(serializers.Serializer):
    messages = serializers.ListField(child=ChatCompletionMessageSerializer(), min_length=1)
    max_tokens = serializers.IntegerField(required=False, min_value=1, max_value=32768)


class ChoiceSerializer(serializers.Serializer):
    index = serializers.IntegerField(default=0)
    message = ChatCompletionMessageSerializer()
    finish_reason = serializers.ChoiceField(choices=["stop", "length"])


class ChatCompletionResultSerializer(serializers.Serializer):
    choices = serializers.ListField(child=ChoiceSerializer())
    usage = serializers.DictField(required=False)


class BotUserSerializer(serializers.ModelSerializer):
    class Meta:
        model = BotUser
        fields = ("user_id", "username", "language")


class BotSerializer(serializers.ModelSerializer):
    class Meta:
        model = Bot
        fields = ["codename"]


class DialogSerializer(serializers.ModelSerializer):
    bot = serializers.SlugRelatedField("codename", queryset=Bot.objects.all(), source="instance.bot")
    user = BotUserSerializer(source="instance.user", required=False)

    class Meta:
        model = Dialog
        fields = ("id", "bot", "user", "is_completed")

    def create(self, validated_data):
        inst = validated_data.pop("instance", {})
        user_data = dict(inst.pop("user", {}) or {})
        dialog_id = uuid.uuid4()
        bot_user, _ = BotUser.objects.get_or_create(user_id=user_data.pop("user_id", str(dialog_id)),
                                                    platform="api", defaults=user_data)
        instance, _ = Instance.objects.get_or_create(bot=inst["bot"], user=bot_user)
        return Dialog.objects.create(id=dialog_id, instance=instance, **validated_data)

    def update(self, instance, validated_data):
        inst = validated_data.pop("instance", {}) or {}
        if "bot" in inst and inst["bot"] != instance.instance.bot:
            new_instance, _ = Instance.objects.get_or_create(bot=inst["bot"], user=instance.instance.user)
            instance.instance = new_instance
        return super().update(instance, validated_data)


class MessageSerializer(serializers.ModelSerializer):
    timestamp = serializers.SerializerMethodField()

    class Meta:
        model = Message
        fields = ("id", "timestamp", "text")

    def get_timestamp(self, obj):
        if isinstance(obj, dict):
            return obj.get("timestamp")
        return int(obj.timestamp.timestamp())


class AnsweredMessageSerializer(MessageSerializer):
    answer = serializers.SerializerMethodField()

    class Meta(MessageSerializer.Meta):
        fields = MessageSerializer.Meta.fields + ("answer",)

    def get_answer(self, obj):
        if isinstance(obj, dict):
            return obj.get("answer")
        replies = Message.objects.filter(dialog_id=obj.dialog_id, role__name="assistant", id__gt=obj.id).order_by("id")
        return MessageSerializer(replies, many=True).data
