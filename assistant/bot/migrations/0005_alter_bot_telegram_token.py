"""Bots without a Telegram token (console / API-only bots)."""
from django.db import migrations

from ._schema import char


class Migration(migrations.Migration):
    dependencies = [("assistant_bot", "0004_message_photo")]

    operations = [migrations.AlterField("bot", "telegram_token", char())]
