"""Photos attached to messages (vision models)."""
from django.db import migrations, models

from ._schema import upgrade_safe


class Migration(migrations.Migration):
    dependencies = [("assistant_bot", "0003_botuser_instance_dialog_message")]

    operations = [
        upgrade_safe(migrations.AddField("message", "photo", models.ImageField(upload_to="photos/", null=True,
                                                                            blank=True))),
    ]
