"""Knowledge-base models (reference storage/models.py:7-87).

``WikiDocument`` is an MPTT tree of wiki pages per bot; ingest splits a page into ``Document``
sections, each with LLM-extracted ``Sentence`` rows and generated ``Question`` rows carrying 768-d
embeddings.  Embeddings persist here (source of truth); similarity search runs in the exact in-HBM
index (``assistant.storage.index``) instead of a pgvector HNSW index, kept in sync by signals.
"""
from django.db import models
from mptt.fields import TreeForeignKey
from mptt.models import MPTTModel

from assistant.storage.fields import VectorField

EMBEDDING_DIM = 768


class Document(models.Model):
    wiki = models.ForeignKey("WikiDocument", on_delete=models.CASCADE, related_name="documents", null=True,
                             blank=True)
    processing = models.ForeignKey("WikiDocumentProcessing", on_delete=models.CASCADE, related_name="documents",
                                   null=True, blank=True)
    name = models.TextField()
    description = models.TextField(default="", blank=True)
    content = models.TextField(default="", blank=True)
    content_embedding = VectorField(dimensions=EMBEDDING_DIM, blank=True, null=True)

    def __str__(self):
        return self.wiki.path.replace(" / ", ". ") if self.wiki_id else self.name


class BaseEmbeddingModel(models.Model):
    document = models.ForeignKey("Document", on_delete=models.CASCADE, related_name="%(class)ss")
    text = models.TextField()
    order = models.PositiveIntegerField(default=0)
    embedding = VectorField(dimensions=EMBEDDING_DIM, blank=True, null=True)

    class Meta:
        abstract = True

    def __str__(self):
        return self.text


class Sentence(BaseEmbeddingModel):
    pass


class Question(BaseEmbeddingModel):
    pass


class WikiDocument(MPTTModel):
    bot = models.ForeignKey("assistant_bot.Bot", on_delete=models.CASCADE, related_name="wikis", null=True,
                            blank=True)
    parent = TreeForeignKey("self", on_delete=models.CASCADE, null=True, blank=True, related_name="children")
    url = models.URLField(blank=True, null=True, verbose_name="URL")
    title = models.TextField(blank=True, verbose_name="Заголовок")
    description = models.TextField(default="", blank=True, verbose_name="Описание")
    content = models.TextField(default="", blank=True, verbose_name="Содержание")
    created_at = models.DateTimeField(auto_now_add=True, verbose_name="Дата создания")
    updated_at = models.DateTimeField(auto_now=True, verbose_name="Дата обновления")

    def __str__(self):
        return f"{self.title}"

    @property
    def path(self) -> str:
        return " / ".join(str(a) for a in self.get_ancestors(include_self=True))


class WikiDocumentProcessing(models.Model):
    class Status(models.TextChoices):
        IN_PROGRESS = "in_progress", "In progress"
        COMPLETED = "completed", "Completed"
        FAILED = "failed", "Failed"

    wiki_document = models.ForeignKey("WikiDocument", on_delete=models.CASCADE, related_name="processing")
    status = models.CharField(max_length=20, choices=Status.choices, default=Status.IN_PROGRESS)
