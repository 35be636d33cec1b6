"""Register the Telegram webhook when a bot's token or callback URL changes
(reference bot/signals.py:14-46)."""
import json
import logging
import urllib.request

from django.db.models.signals import post_save, pre_save
from django.dispatch import receiver

from assistant.bot.models import Bot

logger = logging.getLogger(__name__)


@receiver(pre_save, sender=Bot)
def bot_pre_save(sender, instance, **kwargs):
    instance._original = Bot.objects.filter(pk=instance.pk).first() if instance.pk else None


@receiver(post_save, sender=Bot)
def bot_post_save(sender, instance, created, **kwargs):
    orig = getattr(instance, "_original", None)
    changed = created or orig is None or instance.telegram_token != orig.telegram_token \
        or instance.callback_url != orig.callback_url
    if not changed:
        return
    if instance.telegram_token and instance.callback_url:
        logger.info("Setting webhook %s for bot %s", instance.callback_url, instance.codename)
        set_webhook(instance.telegram_token, instance.callback_url)
    else:
        logger.info("Skipping webhook for bot %s: no token or callback URL", instance.codename)


def set_webhook(token: str, url: str, timeout: float = 30.0):
    req = urllib.request.Request(f"https://api.telegram.org/bot{token}/setWebhook",
                                 data=json.dumps({"url": url}).encode(),
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        body = json.loads(r.read())
    if not body.get("ok"):
        raise RuntimeError(f"Telegram API error: {body}")
    return body
