"""Shared helpers of the bot management commands (reference bot/management/commands/utils.py)."""
from assistant.bot.domain import User
from assistant.bot.models import Bot, BotUser, Instance
from assistant.bot.views import display_username


def get_instance(codename: str, platform_codename: str, chat_id: str, user: User):
    bot, _ = Bot.objects.get_or_create(codename=codename)
    language = user.language_code if user else None
    username = (display_username(user) or "") if user else None
    bot_user, _ = BotUser.objects.get_or_create(user_id=chat_id, platform=platform_codename,
                                                defaults={"username": username, "language": language})
    changed = []
    if bot_user.language != language:
        bot_user.language = language
        changed.append("language")
    if bot_user.username != username:
        bot_user.username = username
        changed.append("username")
    if changed:
        bot_user.save(update_fields=changed)
    instance, _ = Instance.objects.get_or_create(user_id=bot_user.id, bot_id=bot.id)
    return Instance.objects.select_related("bot", "user").get(id=instance.id)
