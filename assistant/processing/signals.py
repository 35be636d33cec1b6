"""Ingest trigger (reference processing/signals.py:8-10): every save of a WikiDocument (re)processes it.
Saves that only touch bookkeeping fields (``update_fields`` without title/content) are skipped."""
from django.db.models.signals import post_save
from django.dispatch import receiver

from assistant.storage.models import WikiDocument

from .tasks import wiki_processing_task

CONTENT_FIELDS = {"title", "content", "description", "parent"}


@receiver(post_save, sender=WikiDocument)
def wiki_document_post_save(sender, instance, created, update_fields=None, **kwargs):
    if update_fields is not None and not (set(update_fields) & CONTENT_FIELDS):
        return
    wiki_processing_task.delay(instance.id)
