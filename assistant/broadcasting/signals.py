"""DRAFT <-> SCHEDULED on scheduled_at changes (reference broadcasting/signals.py:5-48)."""
from django.db.models.signals import pre_save
from django.dispatch import receiver

from assistant.broadcasting import core

from .models import BroadcastCampaign


@receiver(pre_save, sender=BroadcastCampaign)
def update_campaign_status_on_schedule(sender, instance, update_fields=None, **kwargs):
    original = sender.objects.filter(pk=instance.pk).values_list("status", flat=True).first() if instance.pk else None
    instance.status = core.schedule_transition(instance.status, instance.scheduled_at, original, update_fields)
