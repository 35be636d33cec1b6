"""Broadcast campaigns (reference broadcasting/models.py:9-98)."""
from django.db import models
from django.utils.translation import gettext_lazy as _

from assistant.bot.models import Bot
from assistant.broadcasting import core


class BroadcastCampaign(models.Model):
    class Status(models.TextChoices):
        DRAFT = core.DRAFT, _("Draft")
        SCHEDULED = core.SCHEDULED, _("Scheduled")
        SENDING = core.SENDING, _("Sending")
        COMPLETED = core.COMPLETED, _("Completed")
        PARTIAL_FAILURE = core.PARTIAL_FAILURE, _("Partial Failure")
        FAILED = core.FAILED, _("Failed")
        CANCELED = core.CANCELED, _("Canceled")

    class PlatformChoices(models.TextChoices):
        TELEGRAM = "telegram", _("Telegram")

    name = models.CharField(_("Campaign Name"), max_length=255, blank=True, null=True)
    message_text = models.TextField(_("Message Text"))
    bot = models.ForeignKey(Bot, on_delete=models.CASCADE, related_name="broadcast_campaigns", verbose_name=_("Bot"))
    platform = models.CharField(_("Platform"), max_length=20, choices=PlatformChoices.choices,
                                default=PlatformChoices.TELEGRAM)
    status = models.CharField(_("Status"), max_length=20, choices=Status.choices, default=Status.DRAFT,
                              db_index=True)
    scheduled_at = models.DateTimeField(_("Scheduled At"), null=True, blank=True, db_index=True,
                                        help_text=_("Sending starts at this time; leave blank to keep a draft."))
    started_at = models.DateTimeField(_("Started Sending At"), null=True, blank=True)
    completed_at = models.DateTimeField(_("Completed At"), null=True, blank=True)
    total_recipients = models.PositiveIntegerField(_("Total Recipients"), null=True, blank=True)
    successful_sents = models.PositiveIntegerField(_("Successful Sends"), default=0)
    failed_sents = models.PositiveIntegerField(_("Failed Sends"), default=0,
                                               help_text=_("Unavailable users and other delivery errors."))
    created_at = models.DateTimeField(_("Created At"), auto_now_add=True)
    updated_at = models.DateTimeField(_("Updated At"), auto_now=True)

    class Meta:
        verbose_name = _("Broadcast Campaign")
        verbose_name_plural = _("Broadcast Campaigns")
        ordering = ["-scheduled_at", "-created_at"]

    def __str__(self):
        return self.name or f"Campaign for {self.bot.codename} on {self.get_platform_display()} " \
                            f"({self.get_status_display()})"

    def message(self) -> dict:
        """Serialized answer sent to every recipient."""
        return {"text": self.message_text}
