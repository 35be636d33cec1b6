"""Keeps the HBM index in sync with single-row saves / deletes (cascades included), and the rows'
group bits (bot, COMPLETED run) in sync with the wiki they belong to."""
from django.db.models.signals import post_delete, post_save, pre_save
from django.dispatch import receiver

from assistant.storage.index import get_index_service
from assistant.storage.models import Document, Question, Sentence, WikiDocument, WikiDocumentProcessing


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


@receiver(post_save, sender=WikiDocumentProcessing)
def _processing_saved(sender, instance, **kwargs):
    """A run's status changed (finalize, or an admin edit): re-mirror the wiki's completed bit."""
    get_index_service().refresh_wiki(instance.wiki_document_id)


@receiver(pre_save, sender=WikiDocument)
def _wiki_stash_bot(sender, instance, **kwargs):
    old = sender.objects.filter(pk=instance.pk).values_list("bot_id", flat=True).first() if instance.pk else None
    instance._dab_old_bot_id = old


@receiver(post_save, sender=WikiDocument)
def _wiki_saved(sender, instance, created=False, **kwargs):
    """A wiki moved to another bot: its rows change group."""
    if not created and getattr(instance, "_dab_old_bot_id", instance.bot_id) != instance.bot_id:
        get_index_service().refresh_wiki(instance.pk)
