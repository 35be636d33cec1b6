"""Admin site pieces shared by the apps (reference admin/admin.py)."""
from django.contrib import admin
from django.contrib.admin import AdminSite


class AssistantAdminSite(AdminSite):
    site_title = "Bots admin"
    site_header = "Bots admin"
    index_title = ""


class TokenAdmin(admin.ModelAdmin):
    list_display = ("user", "created")
    readonly_fields = ("key", "created")


class SuperUserMixin:
    """Hide a ModelAdmin from non-superusers."""

    def has_module_permission(self, request):
        return request.user.is_superuser
