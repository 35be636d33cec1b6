"""Admin registrations of the example project (reference example/bot/admin.py): the library's model
admins are registered by the apps themselves; here only the token admin is added."""
from django.contrib import admin

from assistant.admin.admin import TokenAdmin

try:
    from rest_framework.authtoken.models import TokenProxy

    admin.site.unregister(TokenProxy)
    admin.site.register(TokenProxy, TokenAdmin)
except Exception:  # authtoken not installed / not registered
    pass
