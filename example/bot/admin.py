"""Admin registrations of the example host (reference example/bot/admin.py:6-9): the library ships
the model admins, the host decides what its admin site shows."""
from django.contrib import admin

from assistant.bot.admin import BotAdmin, DialogAdmin, InstanceAdmin, MessageAdmin
from assistant.bot.models import Bot, Dialog, Instance, Message

admin.site.register(Bot, BotAdmin)
admin.site.register(Instance, InstanceAdmin)
admin.site.register(Dialog, DialogAdmin)
admin.site.register(Message, MessageAdmin)
