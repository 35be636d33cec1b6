"""Celery queue names (reference assistant/assistant/queue.py).  Queries, ingest and broadcasts run
on separate queues so a long document-processing backlog never delays user answers."""
from enum import Enum


class CeleryQueues(Enum):
    QUERY = "query"
    PROCESSING = "processing"
    BROADCASTING = "broadcasting"
