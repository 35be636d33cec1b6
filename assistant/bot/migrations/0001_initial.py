"""First bot schema: per-bot Instances keyed by the platform user id (replaced in 0002/0003)."""
from django.db import migrations

from ._schema import MESSAGE_OPTIONS, char, created, fk, flag, message_fields, pk, state, text


class Migration(migrations.Migration):
    initial = True
    dependencies = []

    operations = [
        migrations.CreateModel("Bot", [
            ("id", pk()),
            ("codename", char(optional=False, unique=True)),
            ("username", char()),
            ("help_text", text()),
            ("start_text", text()),
            ("system_text", text()),
            ("telegram_whitelist", text()),
            ("telegram_token", char(optional=False)),
            ("is_whitelist_enabled", flag()),
        ]),
        migrations.CreateModel("Role", [("id", pk()), ("name", char(optional=False))]),
        migrations.CreateModel("Instance", [
            ("id", pk()),
            ("created_at", created()),
            ("user_id", char(optional=False, db_index=True)),
            ("username", char()),
            ("language", char()),
            ("state", state()),
            ("bot", fk("bot")),
        ]),
        migrations.CreateModel("Dialog", [
            ("id", pk()),
            ("is_completed", flag(indexed=True)),
            ("instance", fk("instance", related_name="dialogs")),
        ]),
        migrations.CreateModel("Message", message_fields(), options=dict(MESSAGE_OPTIONS)),
    ]
