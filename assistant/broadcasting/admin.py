"""Campaign admin with a "send test message" widget (reference broadcasting/admin.py:25-267).

Both test paths send the campaign text as a plain {'text': ...} answer (the reference json-parsed the
text in one path and wrapped it in the other).  Registration is the host's, as in the reference
(``admin.site.register(BroadcastCampaign, BroadcastCampaignAdmin)`` in a host app's admin.py)."""
import json
import logging

from django.contrib import admin, messages
from django.http import HttpRequest, HttpResponseRedirect, JsonResponse
from django.shortcuts import get_object_or_404
from django.urls import path, reverse
from django.utils.decorators import method_decorator
from django.utils.translation import gettext_lazy as _
from django.views.decorators.csrf import csrf_protect

from assistant.bot.domain import answer_from_dict
from assistant.bot.exceptions import UserUnavailableError
from assistant.bot.models import Bot, BotUser
from assistant.bot.utils import get_bot_platform
from assistant.broadcasting import core
from assistant.utils.sync import async_to_sync

from .models import BroadcastCampaign

logger = logging.getLogger(__name__)
EDITABLE_IN_DRAFT = ("scheduled_at", "message_text", "platform", "name", "bot")


def send_test(bot_codename: str, platform_code: str, text: str, username: str) -> str:
    """Deliver ``text`` to the user with ``username`` -> user-facing message; raises on failure."""
    username = username if username.startswith("@") else "@" + username
    user = BotUser.objects.get(platform=platform_code, username=username)
    platform = get_bot_platform(bot_codename, platform_code)
    async_to_sync(core.post_answer)(platform, user.user_id, answer_from_dict({"text": text}))
    return f"Test message sent to {username}."


class BroadcastCampaignAdmin(admin.ModelAdmin):
    list_display = ("__str__", "bot", "platform", "status", "total_recipients", "successful_sents", "failed_sents",
                    "created_at")
    list_filter = ("status", "platform", "bot", "created_at")
    search_fields = ("name", "bot__codename", "message_text")
    readonly_fields = ("status", "started_at", "completed_at", "total_recipients", "successful_sents",
                       "failed_sents", "created_at", "updated_at")
    fieldsets = (
        (None, {"fields": ("name", "bot", "platform", "message_text", "scheduled_at")}),
        (_("Status & Statistics"), {"classes": ("collapse",), "fields": (
            "status", "started_at", "completed_at", "total_recipients", "successful_sents", "failed_sents")}),
        (_("Timestamps"), {"classes": ("collapse",), "fields": ("created_at", "updated_at")}),
    )
    change_form_template = "admin/broadcasting/broadcastcampaign/change_form.html"
    add_form_template = "admin/broadcasting/broadcastcampaign/add_form.html"
    actions = ["cancel_campaigns"]

    def get_changeform_initial_data(self, request):
        initial = super().get_changeform_initial_data(request)
        bots = Bot.objects.all()[:2]
        if len(bots) == 1:
            initial["bot"] = bots[0].pk
        return initial

    def get_readonly_fields(self, request, obj=None):
        ro = list(super().get_readonly_fields(request, obj))
        if obj is not None and obj.status != BroadcastCampaign.Status.DRAFT:
            ro += [f for f in EDITABLE_IN_DRAFT if f not in ro]
        return tuple(ro)

    @admin.action(description=_("Cancel selected draft / scheduled campaigns"))
    def cancel_campaigns(self, request, queryset):
        n = queryset.filter(status__in=[BroadcastCampaign.Status.DRAFT, BroadcastCampaign.Status.SCHEDULED]) \
            .update(status=BroadcastCampaign.Status.CANCELED)
        self.message_user(request, f"{n} campaign(s) canceled.")

    def get_urls(self):
        return [
            path("<int:campaign_id>/send-test/", self.admin_site.admin_view(self.process_send_test),
                 name="broadcasting_broadcastcampaign_send_test"),
            path("ajax-send-test/", self.admin_site.admin_view(self.ajax_send_test_message),
                 name="broadcasting_broadcastcampaign_ajax_send_test"),
        ] + super().get_urls()

    def process_send_test(self, request: HttpRequest, campaign_id: int):
        back = HttpResponseRedirect(reverse("admin:broadcasting_broadcastcampaign_change", args=[campaign_id]))
        campaign = self.get_object(request, str(campaign_id))
        if campaign is None:
            messages.error(request, "Campaign not found.")
            return HttpResponseRedirect(reverse("admin:broadcasting_broadcastcampaign_changelist"))
        if campaign.status != BroadcastCampaign.Status.DRAFT:
            messages.warning(request, "Test messages can only be sent for DRAFT campaigns.")
            return back
        username = (request.POST.get("test_username") or "").strip() if request.method == "POST" else ""
        if not username:
            messages.error(request, "Test username cannot be empty.")
            return back
        try:
            messages.success(request, send_test(campaign.bot.codename, campaign.platform, campaign.message_text,
                                                username))
        except BotUser.DoesNotExist:
            messages.error(request, f"User {username!r} not found on {campaign.platform}.")
        except UserUnavailableError:
            messages.warning(request, f"User {username!r} is unavailable or has blocked the bot.")
        except Exception as e:
            logger.exception("test send failed")
            messages.error(request, f"Unexpected error: {e}")
        return back

    @method_decorator(csrf_protect)
    def ajax_send_test_message(self, request: HttpRequest):
        if request.method != "POST":
            return JsonResponse({"status": "error", "message": "Invalid request method."}, status=405)
        try:
            data = json.loads(request.body or b"{}")
        except json.JSONDecodeError:
            return JsonResponse({"status": "error", "message": "Invalid JSON."}, status=400)
        fields = [data.get(k) for k in ("bot_id", "platform_code", "message_text", "test_username")]
        if not all(fields):
            return JsonResponse({"status": "error", "message": "Missing required data."}, status=400)
        bot_id, platform_code, text, username = fields
        try:
            bot = get_object_or_404(Bot, pk=int(bot_id))
            return JsonResponse({"status": "success", "message": send_test(bot.codename, platform_code, text,
                                                                           username)})
        except (ValueError, TypeError):
            return JsonResponse({"status": "error", "message": "Invalid Bot ID."}, status=400)
        except BotUser.DoesNotExist:
            return JsonResponse({"status": "error", "message": f"User {username!r} not found."}, status=404)
        except UserUnavailableError:
            return JsonResponse({"status": "warning", "message": f"User {username!r} is unavailable."}, status=400)
        except Exception as e:
            logger.exception("ajax test send failed")
            return JsonResponse({"status": "error", "message": f"Unexpected error: {e}"}, status=500)

    def change_view(self, request, object_id, form_url="", extra_context=None):
        extra_context = extra_context or {}
        campaign = self.get_object(request, object_id)
        if campaign is not None and campaign.status == BroadcastCampaign.Status.DRAFT:
            extra_context["show_test_send"] = True
            extra_context["test_send_url"] = reverse("admin:broadcasting_broadcastcampaign_send_test",
                                                     args=[campaign.pk])
        return super().change_view(request, object_id, form_url, extra_context=extra_context)

    def add_view(self, request, form_url="", extra_context=None):
        extra_context = extra_context or {}
        extra_context["ajax_test_send_url"] = reverse("admin:broadcasting_broadcastcampaign_ajax_send_test")
        return super().add_view(request, form_url, extra_context=extra_context)
