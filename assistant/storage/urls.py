from django.urls import include, path
from rest_framework.routers import DefaultRouter

from assistant.storage.api.views import WikiDocumentViewSet

router = DefaultRouter()
router.register(r"documents", WikiDocumentViewSet)

urlpatterns = [path("", include(router.urls))]
