"""Django settings for the (optional) Django integration tests: SQLite, eager Celery, fake AI
(reference tests/settings.py, which required PostgreSQL).  Used by tests/django_tests/ when Django,
DRF and django-mptt are installed; skipped otherwise."""
import os
import tempfile

SECRET_KEY = "tests"
DEBUG = True
ALLOWED_HOSTS = ["*"]
USE_TZ = False
DATABASES = {"default": {"ENGINE": "django.db.backends.sqlite3",
                         "NAME": os.path.join(tempfile.gettempdir(), "dab_tests.sqlite3")}}
INSTALLED_APPS = [
    "django.contrib.admin", "django.contrib.auth", "django.contrib.contenttypes", "django.contrib.sessions",
    "django.contrib.messages", "rest_framework", "rest_framework.authtoken", "mptt",
    "assistant.bot", "assistant.storage", "assistant.processing", "assistant.rag", "assistant.broadcasting",
    "assistant.admin",
]
MIDDLEWARE = ["django.contrib.sessions.middleware.SessionMiddleware",
              "django.contrib.auth.middleware.AuthenticationMiddleware",
              "django.contrib.messages.middleware.MessageMiddleware"]
ROOT_URLCONF = "assistant.assistant.urls"
TEMPLATES = [{"BACKEND": "django.template.backends.django.DjangoTemplates", "APP_DIRS": True,
              "OPTIONS": {"context_processors": ["django.contrib.auth.context_processors.auth",
                                                 "django.contrib.messages.context_processors.messages",
                                                 "django.template.context_processors.request"]}}]
REST_FRAMEWORK = {"DEFAULT_AUTHENTICATION_CLASSES": ["rest_framework.authentication.TokenAuthentication"],
                  "DEFAULT_PERMISSION_CLASSES": ["rest_framework.permissions.IsAuthenticated"]}
DEFAULT_AUTO_FIELD = "django.db.models.BigAutoField"
DEFAULT_AI_MODEL = "test"
EMBEDDING_AI_MODEL = "test"
VECTOR_INDEX_BACKEND = "db"
CELERY_TASK_ALWAYS_EAGER = True
BOTS = {"default": {}}
RESOURCES_DIR = os.path.join(os.path.dirname(__file__), "resources")
