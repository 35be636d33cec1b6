"""Django admin for bots, dialogs, instances and messages (reference bot/admin.py).

The classes are not registered here: as in the reference (whose ``@admin.register`` lines are
commented out, reference bot/admin.py:19,37,63,104), the host project registers them
(reference example/bot/admin.py:6-9 ``admin.site.register(Bot, BotAdmin)`` ...); registering them
here too would make the host's registration raise ``AlreadyRegistered``."""
from django import forms
from django.contrib import admin
from django.db import models
from django.urls import reverse
from django.utils.html import format_html

from assistant.bot.models import Bot, Dialog, Instance, Message


class BotAdminForm(forms.ModelForm):
    telegram_token = forms.CharField(widget=forms.PasswordInput(render_value=True), required=False)

    class Meta:
        model = Bot
        fields = "__all__"


class BotAdmin(admin.ModelAdmin):
    form = BotAdminForm
    list_display = ["codename", "is_whitelist_enabled"]
    search_fields = ["codename"]
    readonly_fields = ["callback_url"]
    exclude = ["username"]

    @admin.display(description="Telegram callback URL")
    def callback_url(self, obj):
        return obj.callback_url


class DialogAdmin(admin.ModelAdmin):
    list_display = ("id", "bot_link", "instance_link", "is_completed", "messages_link")
    list_filter = ["is_completed", "instance__bot__codename"]
    list_select_related = ("instance", "instance__bot", "instance__user")

    @admin.display(description="Bot")
    def bot_link(self, obj):
        url = reverse("admin:assistant_bot_bot_change", args=[obj.instance.bot_id])
        return format_html('<a href="{}">{}</a>', url, obj.instance.bot.codename)

    @admin.display(description="Instance")
    def instance_link(self, obj):
        url = reverse("admin:assistant_bot_instance_change", args=[obj.instance_id])
        return format_html('<a href="{}">{}</a>', url, obj.instance.user.username or obj.instance.user.user_id)

    @admin.display(description="Messages")
    def messages_link(self, obj):
        url = reverse("admin:assistant_bot_message_changelist")
        n = Message.objects.filter(dialog_id=obj.id).count()
        return format_html('<a href="{}?dialog__id__exact={}">View messages ({})</a>', url, obj.id, n)


class InstanceAdmin(admin.ModelAdmin):
    list_display = ("username_display", "bot_link", "created_at", "is_unavailable", "total_cost")
    search_fields = ["user__username", "bot__codename"]
    list_filter = ["bot__codename", "is_unavailable", "created_at"]
    readonly_fields = ["created_at"]

    def get_queryset(self, request):
        return super().get_queryset(request).select_related("bot", "user").annotate(
            _total_cost=models.Sum("dialogs__messages__cost"))

    @admin.display(description="Username")
    def username_display(self, obj):
        return obj.user.username

    @admin.display(description="Bot")
    def bot_link(self, obj):
        url = reverse("admin:assistant_bot_bot_change", args=[obj.bot_id])
        return format_html('<a href="{}">{}</a>', url, obj.bot.codename)

    @admin.display(description="Cost", ordering="_total_cost")
    def total_cost(self, obj):
        return obj._total_cost


class MessageAdmin(admin.ModelAdmin):
    list_display = ["timestamp", "dialog_link", "role", "short_text", "io_tokens"]
    search_fields = ["text", "role__name"]
    list_filter = ["role", "timestamp", "dialog__instance__bot__codename"]
    readonly_fields = ["full_text", "message_id", "timestamp", "dialog", "role"]
    exclude = ["text", "cost"]
    list_select_related = ("dialog", "dialog__instance", "dialog__instance__bot", "role")

    @admin.display(description="Bot (dialog)")
    def dialog_link(self, obj):
        url = reverse("admin:assistant_bot_dialog_change", args=[obj.dialog_id])
        return format_html('{} (<a href="{}">{}</a>)', obj.dialog.instance.bot.codename, url, obj.dialog_id)

    @admin.display(description="Text")
    def short_text(self, obj):
        if obj.text and len(obj.text) > 85:
            return f"{obj.text[:80]}... ({len(obj.text)} chars)"
        return obj.text

    @admin.display(description="Text")
    def full_text(self, obj):
        return obj.text

    @admin.display(description="I/O tokens")
    def io_tokens(self, obj):
        if obj.cost_details:
            last = obj.cost_details[-1]
            return f"{last.get('prompt_tokens', '-')} / {last.get('completion_tokens', '-')}"

    def lookup_allowed(self, lookup, value, request=None):
        if lookup in ("dialog__instance__id__exact", "dialog__id__exact"):
            return True
        return super().lookup_allowed(lookup, value, request) if request is not None \
            else super().lookup_allowed(lookup, value)
