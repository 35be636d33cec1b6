"""Platform users (BotUser) and the current Instance / Dialog (UUID ids) / Message tables."""
from django.db import migrations

from ._schema import MESSAGE_OPTIONS, char, created, fk, flag, message_fields, pk, state, upgrade_safe, uuid_pk


class Migration(migrations.Migration):
    dependencies = [("assistant_bot", "0002_remove_dialog_and_message_and_instance")]

    operations = [
        upgrade_safe(migrations.CreateModel("BotUser", [
            ("id", pk()),
            ("created_at", created()),
            ("user_id", char(optional=False)),
            ("platform", char(optional=False)),
            ("username", char()),
            ("language", char()),
        ], options={"unique_together": {("user_id", "platform")}})),
        upgrade_safe(migrations.CreateModel("Instance", [
            ("id", pk()),
            ("created_at", created()),
            ("state", state()),
            ("bot", fk("bot")),
            ("user", fk("botuser")),
        ])),
        upgrade_safe(migrations.CreateModel("Dialog", [
            ("id", uuid_pk()),
            ("created_at", created()),
            ("is_completed", flag(indexed=True)),
            ("state", state()),
            ("instance", fk("instance", related_name="dialogs")),
        ])),
        upgrade_safe(migrations.CreateModel("Message", message_fields(), options=dict(MESSAGE_OPTIONS))),
    ]
