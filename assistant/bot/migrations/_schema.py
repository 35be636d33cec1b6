"""Field factories for the bot app's migration chain (Django's loader skips ``_``-prefixed modules).

The chain keeps the reference's migration names (assistant/bot/migrations/0001-0006 there), so a
database created by the reference upgrades in place; a fresh database replays the same history."""
import uuid

from django.db import models
from django.db.models import deletion


def pk():
    return models.BigAutoField(auto_created=True, primary_key=True, serialize=False, verbose_name="ID")


def uuid_pk():
    return models.UUIDField(default=uuid.uuid4, editable=False, primary_key=True, serialize=False)


def char(n=100, optional=True, **kw):
    return models.CharField(max_length=n, null=optional, blank=optional, **kw) if optional else \
        models.CharField(max_length=n, **kw)


def text():
    return models.TextField(null=True, blank=True)


def created():
    return models.DateTimeField(auto_now_add=True)


def state():
    return models.JSONField(default=dict, blank=True)


def flag(indexed=False):
    return models.BooleanField(default=False, db_index=True) if indexed else models.BooleanField(default=False)


def fk(model, **kw):
    return models.ForeignKey(on_delete=deletion.CASCADE, to=f"assistant_bot.{model}", **kw)


def message_fields(with_photo=False):
    fields = [
        ("id", pk()),
        ("timestamp", created()),
        ("message_id", models.BigIntegerField(db_index=True, null=True, blank=True)),
        ("text", text()),
    ]
    if with_photo:
        fields.append(("photo", models.ImageField(upload_to="photos/", null=True, blank=True)))
    fields += [
        ("cost_details", state()),
        ("cost", models.DecimalField(max_digits=16, decimal_places=8, null=True, blank=True)),
        ("dialog", fk("dialog", related_name="messages")),
        ("role", fk("role")),
    ]
    return fields


MESSAGE_OPTIONS = {"unique_together": {("dialog", "message_id")}}
