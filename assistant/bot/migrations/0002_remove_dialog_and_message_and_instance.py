"""Drops the first conversation tables (users become platform-scoped BotUsers in 0003)."""
from django.db import migrations

from ._schema import upgrade_safe


class Migration(migrations.Migration):
    dependencies = [("assistant_bot", "0001_initial")]

    # upgrade_safe: a database that already holds the final tables keeps them (see _schema.py)
    operations = [upgrade_safe(migrations.DeleteModel(name)) for name in ("Message", "Dialog", "Instance")]
