import django.db.models.deletion
import mptt.fields
from django.db import migrations, models

import assistant.storage.fields


class Migration(migrations.Migration):
    """Knowledge-base schema.  Vectors use the portable VectorField (pgvector type on PostgreSQL when
    pgvector is installed, float32 bytes elsewhere); no HNSW index -- search runs in the HBM index.
    Document.content_embedding and the WikiDocument verbose names follow in 0002 (the reference's
    migration names, so a database it created continues from its own history)."""

    initial = True

    dependencies = [
        ("assistant_bot", "0001_initial"),
    ]

    operations = [
        migrations.CreateModel(
            name="WikiDocument",
            fields=[
                ("id", models.BigAutoField(auto_created=True, primary_key=True, serialize=False, verbose_name="ID")),
                ("url", models.URLField(blank=True, null=True)),
                ("title", models.TextField(blank=True)),
                ("description", models.TextField(blank=True, default="")),
                ("content", models.TextField(blank=True, default="")),
                ("created_at", models.DateTimeField(auto_now_add=True)),
                ("updated_at", models.DateTimeField(auto_now=True)),
                ("lft", models.PositiveIntegerField(editable=False)),
                ("rght", models.PositiveIntegerField(editable=False)),
                ("tree_id", models.PositiveIntegerField(db_index=True, editable=False)),
                ("level", models.PositiveIntegerField(editable=False)),
                ("bot", models.ForeignKey(blank=True, null=True, on_delete=django.db.models.deletion.CASCADE,
                                          related_name="wikis", to="assistant_bot.bot")),
                ("parent", mptt.fields.TreeForeignKey(blank=True, null=True,
                                                      on_delete=django.db.models.deletion.CASCADE,
                                                      related_name="children", to="assistant_storage.wikidocument")),
            ],
            options={"abstract": False},
        ),
        migrations.CreateModel(
            name="WikiDocumentProcessing",
            fields=[
                ("id", models.BigAutoField(auto_created=True, primary_key=True, serialize=False, verbose_name="ID")),
                ("status", models.CharField(choices=[("in_progress", "In progress"), ("completed", "Completed"),
                                                     ("failed", "Failed")], default="in_progress", max_length=20)),
                ("wiki_document", models.ForeignKey(on_delete=django.db.models.deletion.CASCADE,
                                                    related_name="processing", to="assistant_storage.wikidocument")),
            ],
        ),
        migrations.CreateModel(
            name="Document",
            fields=[
                ("id", models.BigAutoField(auto_created=True, primary_key=True, serialize=False, verbose_name="ID")),
                ("name", models.TextField()),
                ("description", models.TextField(blank=True, default="")),
                ("content", models.TextField(blank=True, default="")),
                ("processing", models.ForeignKey(blank=True, null=True, on_delete=django.db.models.deletion.CASCADE,
                                                 related_name="documents",
                                                 to="assistant_storage.wikidocumentprocessing")),
                ("wiki", models.ForeignKey(blank=True, null=True, on_delete=django.db.models.deletion.CASCADE,
                                           related_name="documents", to="assistant_storage.wikidocument")),
            ],
        ),
        migrations.CreateModel(
            name="Question",
            fields=[
                ("id", models.BigAutoField(auto_created=True, primary_key=True, serialize=False, verbose_name="ID")),
                ("text", models.TextField()),
                ("order", models.PositiveIntegerField(default=0)),
                ("embedding", assistant.storage.fields.VectorField(blank=True, dimensions=768, null=True)),
                ("document", models.ForeignKey(on_delete=django.db.models.deletion.CASCADE, related_name="questions",
                                               to="assistant_storage.document")),
            ],
            options={"abstract": False},
        ),
        migrations.CreateModel(
            name="Sentence",
            fields=[
                ("id", models.BigAutoField(auto_created=True, primary_key=True, serialize=False, verbose_name="ID")),
                ("text", models.TextField()),
                ("order", models.PositiveIntegerField(default=0)),
                ("embedding", assistant.storage.fields.VectorField(blank=True, dimensions=768, null=True)),
                ("document", models.ForeignKey(on_delete=django.db.models.deletion.CASCADE, related_name="sentences",
                                               to="assistant_storage.document")),
            ],
            options={"abstract": False},
        ),
    ]
