"""User phone numbers and the per-instance "unavailable" flag (blocked bot, skipped by broadcasts)."""
from django.db import migrations

from ._schema import char, flag


class Migration(migrations.Migration):
    dependencies = [("assistant_bot", "0005_alter_bot_telegram_token")]

    operations = [
        migrations.AddField("botuser", "phone_number", char(20)),
        migrations.AddField("instance", "is_unavailable", flag(indexed=True)),
    ]
