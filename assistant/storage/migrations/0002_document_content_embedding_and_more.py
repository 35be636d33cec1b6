"""Whole-document embeddings and the Russian admin labels of WikiDocument."""
from django.db import migrations, models

import assistant.storage.fields
from assistant.bot.migrations._schema import upgrade_safe

LABELS = {
    "url": (models.URLField, {"blank": True, "null": True}, "URL"),
    "title": (models.TextField, {"blank": True}, "Заголовок"),
    "description": (models.TextField, {"blank": True, "default": ""}, "Описание"),
    "content": (models.TextField, {"blank": True, "default": ""}, "Содержание"),
    "created_at": (models.DateTimeField, {"auto_now_add": True}, "Дата создания"),
    "updated_at": (models.DateTimeField, {"auto_now": True}, "Дата обновления"),
}


class Migration(migrations.Migration):
    dependencies = [("assistant_storage", "0001_initial")]

    operations = [
        # upgrade_safe: databases of an earlier revision already have the column (bot _schema.py)
        upgrade_safe(migrations.AddField("document", "content_embedding",
                                         assistant.storage.fields.VectorField(blank=True, dimensions=768, null=True))),
    ] + [
        migrations.AlterField("wikidocument", name, cls(verbose_name=label, **kw))
        for name, (cls, kw, label) in LABELS.items()
    ]
