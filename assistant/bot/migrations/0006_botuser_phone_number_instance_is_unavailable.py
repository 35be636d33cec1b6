"""User phone numbers and the per-instance "unavailable" flag (blocked bot, skipped by broadcasts)."""
from django.db import migrations

from ._schema import char, flag, upgrade_safe


class Migration(migrations.Migration):
    dependencies = [("assistant_bot", "0005_alter_bot_telegram_token")]

    operations = [
        upgrade_safe(migrations.AddField("botuser", "phone_number", char(20))),
        upgrade_safe(migrations.AddField("instance", "is_unavailable", flag(indexed=True))),
    ]
