"""Documents REST serializers (reference storage/api/serializers.py).  The processing serializer
exposes the run's ``status`` (the reference named a non-existent ``completed`` field)."""
import calendar

from rest_framework import serializers

from assistant.bot.models import Bot
from assistant.storage.models import WikiDocument, WikiDocumentProcessing


class UnixTimestampField(serializers.DateTimeField):
    def to_representation(self, value):
        return int(calendar.timegm(value.utctimetuple())) if value else None


class WikiDocumentProcessingSerializer(serializers.ModelSerializer):
    completed = serializers.SerializerMethodField()

    class Meta:
        model = WikiDocumentProcessing
        fields = ["id", "status", "completed"]

    def get_completed(self, obj):
        return obj.status == WikiDocumentProcessing.Status.COMPLETED


class WikiDocumentSerializer(serializers.ModelSerializer):
    bot = serializers.CharField(source="bot.codename", required=False)
    created_at = UnixTimestampField(read_only=True)
    updated_at = UnixTimestampField(read_only=True)
    processing = serializers.SerializerMethodField()

    class Meta:
        model = WikiDocument
        exclude = ["lft", "rght", "tree_id", "level"]

    def get_processing(self, obj):
        runs = list(obj.processing.all())
        last = max(runs, key=lambda r: r.id) if runs else None
        return WikiDocumentProcessingSerializer(last).data if last else None

    def create(self, validated_data):
        return super().create(self._set_bot(validated_data))

    def update(self, instance, validated_data):
        return super().update(instance, self._set_bot(validated_data))

    @staticmethod
    def _set_bot(validated_data):
        codename = validated_data.pop("bot", {}).get("codename")
        if codename:
            try:
                validated_data["bot"] = Bot.objects.get(codename=codename)
            except Bot.DoesNotExist:
                raise serializers.ValidationError({"bot": "Bot does not exist."})
        return validated_data
