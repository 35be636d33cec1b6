"""Photos attached to messages (vision models)."""
from django.db import migrations, models


class Migration(migrations.Migration):
    dependencies = [("assistant_bot", "0003_botuser_instance_dialog_message")]

    operations = [
        migrations.AddField("message", "photo", models.ImageField(upload_to="photos/", null=True, blank=True)),
    ]
