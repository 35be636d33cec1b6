from django.apps import AppConfig


class AdminToolsConfig(AppConfig):
    default_auto_field = "django.db.models.BigAutoField"
    name = "assistant.admin"
    label = "assistant_admin"
