"""Ingest Celery tasks on the ``processing`` queue (reference processing/tasks.py:15-74).

wiki_processing_task: split the page (LLM), then fan out one document_processing_task per section and
fan in with finalize_document_processing_task (Celery chain(group, finalize)); finalize marks the run
COMPLETED and deletes older runs of the same page (cascading to their documents / sentences /
questions, whose index rows the storage signals drop).  Without Celery the same phases run inline."""
from __future__ import annotations

import logging

from assistant.assistant.queue import CeleryQueues
from assistant.utils.sync import async_to_sync
from assistant.utils.tasks import HAVE_CELERY, shared_task

logger = logging.getLogger(__name__)

RETRY = dict(queue=CeleryQueues.PROCESSING.value, acks_late=True, autoretry_for=(Exception,),
             reject_on_worker_lost=True, max_retries=10, default_retry_delay=60)


def _repo():
    from assistant.processing.repository import DjangoIngestRepository
    return DjangoIngestRepository()


@shared_task(**RETRY)
def wiki_processing_task(wiki_document_id: int, **kwargs):
    from assistant.processing.wiki import split_wiki_document
    from assistant.storage.models import WikiDocument

    wiki = WikiDocument.objects.filter(id=wiki_document_id).first()
    if wiki is None:
        logger.error("wiki document %s not found", wiki_document_id)
        return
    processing = async_to_sync(split_wiki_document)(wiki, _repo())
    doc_ids = list(processing.documents.values_list("id", flat=True))
    if HAVE_CELERY:
        from celery import chain, group
        chain(group(document_processing_task.si(d) for d in doc_ids),
              finalize_document_processing_task.si(processing.id))()
    else:
        for d in doc_ids:
            document_processing_task(d)
        finalize_document_processing_task(processing.id)


@shared_task(**RETRY)
def document_processing_task(document_id: int, **kwargs):
    from assistant.processing.documents.processor import process_document
    from assistant.storage.models import Document

    document = Document.objects.select_related("wiki", "wiki__bot").get(id=document_id)
    async_to_sync(process_document)(document, _repo())


@shared_task(**RETRY)
def finalize_document_processing_task(processing_id: int, **kwargs):
    from assistant.storage.models import WikiDocumentProcessing

    processing = WikiDocumentProcessing.objects.select_related("wiki_document").get(id=processing_id)
    async_to_sync(_repo().finalize)(processing)
