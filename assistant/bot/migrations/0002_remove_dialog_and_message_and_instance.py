"""Drops the first conversation tables (users become platform-scoped BotUsers in 0003)."""
from django.db import migrations


class Migration(migrations.Migration):
    dependencies = [("assistant_bot", "0001_initial")]

    operations = [migrations.DeleteModel(name) for name in ("Message", "Dialog", "Instance")]
