from django.apps import AppConfig


class StorageConfig(AppConfig):
    default_auto_field = "django.db.models.BigAutoField"
    name = "assistant.storage"
    label = "assistant_storage"

    def ready(self):
        from assistant.storage import signals  # noqa: F401  (keeps the HBM index in sync with the ORM)
