"""Example project settings (reference example/example/settings.py).

Configuration comes from the environment (a ``.env`` file is read when django-environ is installed).
Everything has a working default so ``manage.py migrate && manage.py chat task_manager`` runs on a
laptop with SQLite and the fake AI provider; production points DATABASE_URL at PostgreSQL, the broker
at Redis and the models at the MI355X engine (``engine:llama-3-8b``) or gpu_service."""
import os
from pathlib import Path

BASE_DIR = Path(__file__).resolve().parent.parent
RESOURCES_DIR = BASE_DIR / "bot" / "resources"

try:
    import environ

    ENV = environ.Env()
    environ.Env.read_env(os.path.join(BASE_DIR, ".env"))
except ImportError:  # plain os.environ
    ENV = None


def env(name, default=None):
    return os.environ.get(name, default)


SECRET_KEY = env("SECRET_KEY", "dev-only-not-secret")
DEBUG = env("DEBUG", "0") in ("1", "true", "True")
ALLOWED_HOSTS = env("ALLOWED_HOSTS", "localhost,127.0.0.1").split(",")
TELEGRAM_BASE_CALLBACK_URL = env("TELEGRAM_BASE_CALLBACK_URL")

if env("DATABASE_URL") and ENV is not None:
    DATABASES = {"default": ENV.db("DATABASE_URL")}
else:
    DATABASES = {"default": {"ENGINE": "django.db.backends.sqlite3", "NAME": BASE_DIR / "db.sqlite3"}}

# AI models: "test" (offline fake), "engine:<preset or checkpoint>" (in-process MI355X engine),
# "gpu_service:<model>", "groq:<model>", "ollama:<model>", or an OpenAI model name
DEFAULT_AI_MODEL = env("DEFAULT_AI_MODEL", "test")
DIALOG_FAST_AI_MODEL = env("DIALOG_FAST_AI_MODEL", DEFAULT_AI_MODEL)
DIALOG_STRONG_AI_MODEL = env("DIALOG_STRONG_AI_MODEL", DEFAULT_AI_MODEL)
EMBEDDING_AI_MODEL = env("EMBEDDING_AI_MODEL", "test")
OPENAI_API_KEY = env("OPENAI_API_KEY", "")
GROQ_API_KEY = env("GROQ_API_KEY", "")
GPU_SERVICE_ENDPOINT = env("GPU_SERVICE_ENDPOINT", "http://127.0.0.1:11435")
VECTOR_INDEX_BACKEND = env("VECTOR_INDEX_BACKEND", "engine")  # engine | gpu_service | db

CELERY_BROKER_URL = env("CELERY_BROKER_URL", "redis://127.0.0.1:6379/0")
CELERY_RESULT_BACKEND = CELERY_BROKER_URL
CELERY_ACCEPT_CONTENT = ["json"]
CELERY_TASK_SERIALIZER = "json"
CELERY_TASK_ALWAYS_EAGER = env("CELERY_TASK_ALWAYS_EAGER", "0") == "1"
CELERY_CONCURRENCY = int(env("CELERY_CONCURRENCY", "1"))
try:
    from celery.schedules import crontab

    CELERY_BEAT_SCHEDULE = {"broadcast-campaigns": {"task": "broadcasting.check_scheduled_broadcasts",
                                                    "schedule": crontab(minute="*")}}
except ImportError:
    CELERY_BEAT_SCHEDULE = {}

BOTS = {
    "task_manager": {
        "class": "bot.bot.TaskManagerBot",
        "telegram_token": env("TASK_MANAGER_BOT_TOKEN"),
    },
}

INSTALLED_APPS = [
    "django.contrib.admin",
    "django.contrib.auth",
    "django.contrib.contenttypes",
    "django.contrib.sessions",
    "django.contrib.messages",
    "django.contrib.staticfiles",
    "rest_framework",
    "rest_framework.authtoken",
    "mptt",
    "bot",
    "assistant.bot",
    "assistant.storage",
    "assistant.loading",
    "assistant.processing",
    "assistant.rag",
    "assistant.broadcasting",
    "assistant.admin",
]

MIDDLEWARE = [
    "django.middleware.security.SecurityMiddleware",
    "django.contrib.sessions.middleware.SessionMiddleware",
    "django.middleware.common.CommonMiddleware",
    "django.middleware.csrf.CsrfViewMiddleware",
    "django.contrib.auth.middleware.AuthenticationMiddleware",
    "django.contrib.messages.middleware.MessageMiddleware",
    "django.middleware.clickjacking.XFrameOptionsMiddleware",
    "assistant.assistant.middleware.MediaURLMiddleware",
]

ROOT_URLCONF = "example.urls"
TEMPLATES = [{
    "BACKEND": "django.template.backends.django.DjangoTemplates",
    "DIRS": [],
    "APP_DIRS": True,
    "OPTIONS": {"context_processors": [
        "django.template.context_processors.debug", "django.template.context_processors.request",
        "django.contrib.auth.context_processors.auth", "django.contrib.messages.context_processors.messages"]},
}]
WSGI_APPLICATION = "example.wsgi.application"
ASGI_APPLICATION = "example.asgi.application"

REST_FRAMEWORK = {
    "DEFAULT_AUTHENTICATION_CLASSES": ["rest_framework.authentication.TokenAuthentication",
                                       "rest_framework.authentication.SessionAuthentication"],
    "DEFAULT_PERMISSION_CLASSES": ["rest_framework.permissions.IsAuthenticated"],
    "DEFAULT_PAGINATION_CLASS": "rest_framework.pagination.PageNumberPagination",
    "PAGE_SIZE": 50,
}

LANGUAGE_CODE = "en-us"
TIME_ZONE = "UTC"
USE_I18N = True
USE_TZ = True
STATIC_URL = "static/"
STATIC_ROOT = BASE_DIR / "static"
MEDIA_URL = "/media/"
MEDIA_ROOT = BASE_DIR / "media"
DEFAULT_AUTO_FIELD = "django.db.models.BigAutoField"

LOGGING = {
    "version": 1,
    "disable_existing_loggers": False,
    "formatters": {"plain": {"format": "%(asctime)s %(levelname)s %(name)s: %(message)s"}},
    "handlers": {"console": {"class": "logging.StreamHandler", "formatter": "plain"}},
    "root": {"handlers": ["console"], "level": env("LOG_LEVEL", "INFO")},
    "loggers": {"django.db.backends": {"level": "WARNING"}},
}
