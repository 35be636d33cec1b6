"""Celery app of the example project (reference example/example/celery.py)."""
import logging
import os

from celery import Celery
from celery.signals import setup_logging

os.environ.setdefault("DJANGO_SETTINGS_MODULE", "example.settings")

app = Celery("example")
app.config_from_object("django.conf:settings", namespace="CELERY")
app.conf.worker_concurrency = int(os.environ.get("CELERY_CONCURRENCY", "1"))
app.conf.task_track_started = True
app.autodiscover_tasks()


@setup_logging.connect
def config_loggers(*args, **kwargs):
    from logging.config import dictConfig

    from django.conf import settings

    dictConfig(settings.LOGGING)
    logging.getLogger(__name__).info("celery logging configured")
