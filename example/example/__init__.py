try:  # make the Celery app load with Django (standard Celery/Django wiring)
    from .celery import app as celery_app  # noqa: F401
except ImportError:  # Celery is optional for the console / API
    celery_app = None
