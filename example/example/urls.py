"""URLs of the example project (reference example/example/urls.py)."""
from django.contrib import admin
from django.urls import include, path

urlpatterns = [
    path("admin/", admin.site.urls),
    path("", include("assistant.assistant.urls")),
]
