"""Keeps the HBM index in sync with single-row saves / deletes (cascades included)."""
from django.db.models.signals import post_delete, post_save
from django.dispatch import receiver

from assistant.storage.index import get_index_service
from assistant.storage.models import Document, Question, Sentence


@receiver(post_save, sender=Question)
@receiver(post_save, sender=Sentence)
def _embedding_saved(sender, instance, **kwargs):
    if instance.embedding is not None:
        get_index_service().upsert_objects(sender, [instance], "embedding")


@receiver(post_save, sender=Document)
def _document_saved(sender, instance, **kwargs):
    if instance.content_embedding is not None:
        get_index_service().upsert_objects(sender, [instance], "content_embedding")


@receiver(post_delete, sender=Question)
@receiver(post_delete, sender=Sentence)
def _embedding_deleted(sender, instance, **kwargs):
    get_index_service().remove(sender, [instance.pk], "embedding")


@receiver(post_delete, sender=Document)
def _document_deleted(sender, instance, **kwargs):
    get_index_service().remove(sender, [instance.pk], "content_embedding")
