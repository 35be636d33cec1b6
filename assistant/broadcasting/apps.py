from django.apps import AppConfig


class BroadcastingConfig(AppConfig):
    default_auto_field = "django.db.models.BigAutoField"
    name = "assistant.broadcasting"
    label = "broadcasting"
    verbose_name = "Broadcasting"

    def ready(self):
        from . import signals  # noqa: F401
