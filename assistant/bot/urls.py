"""REST routes of the conversation API (reference bot/urls.py).  Nested message routes are built by
hand so ``drf-nested-routers`` is not required."""
from django.urls import include, path
from rest_framework.routers import DefaultRouter

from assistant.bot.api.views import BotViewSet, DialogViewSet, MessageViewSet

router = DefaultRouter()
router.register(r"bots", BotViewSet)
router.register(r"dialogs", DialogViewSet, basename="dialog")

message_list = MessageViewSet.as_view({"get": "list", "post": "create"})
message_detail = MessageViewSet.as_view({"get": "retrieve"})

urlpatterns = [
    path("", include(router.urls)),
    path("dialogs/<uuid:dialog_pk>/messages/", message_list, name="dialog-messages-list"),
    path("dialogs/<uuid:dialog_pk>/messages/<int:pk>/", message_detail, name="dialog-messages-detail"),
]
