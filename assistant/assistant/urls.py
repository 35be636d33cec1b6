"""Root URL configuration (reference assistant/assistant/urls.py): Telegram webhooks, the REST API of
the installed apps, and (when drf-yasg is installed) Swagger / ReDoc."""
from django.conf import settings
from django.urls import include, path

from assistant.bot.views import TelegramAssistantBotView

urlpatterns = [
    path("telegram/<str:codename>/", TelegramAssistantBotView.as_view(), name="telegram_bot"),
]

try:  # optional API docs
    from drf_yasg import openapi
    from drf_yasg.generators import OpenAPISchemaGenerator
    from drf_yasg.views import get_schema_view
    from rest_framework import permissions
    from rest_framework.authentication import TokenAuthentication

    class BothHttpAndHttpsSchemaGenerator(OpenAPISchemaGenerator):
        def get_schema(self, request=None, public=False):
            schema = super().get_schema(request, public)
            schema.schemes = ["https", "http"]
            return schema

    schema_view = get_schema_view(
        openapi.Info(title="Assistant API", default_version="v1", description="API of the AI assistant"),
        generator_class=BothHttpAndHttpsSchemaGenerator, public=True,
        permission_classes=[permissions.AllowAny], authentication_classes=[TokenAuthentication])
    urlpatterns += [
        path("api/swagger/", schema_view.with_ui("swagger", cache_timeout=0), name="schema-swagger-ui"),
        path("api/redoc/", schema_view.with_ui("redoc", cache_timeout=0), name="schema-redoc"),
    ]
except ImportError:
    pass

if "assistant.storage" in settings.INSTALLED_APPS:
    urlpatterns.append(path("api/v1/", include("assistant.storage.urls")))
if "assistant.bot" in settings.INSTALLED_APPS:
    urlpatterns.append(path("api/v1/", include("assistant.bot.urls")))
if "assistant.rag" in settings.INSTALLED_APPS:
    urlpatterns.append(path("api/v1/", include("assistant.rag.urls")))
