"""LLM self-play QA (reference bot/management/commands/tester.py).

  manage.py tester run <bot> [-n 10]   generate dialogs into test_dialogs/dialog_N.json
  manage.py tester analyze <bot>       review them, write analysis_results.jsonl, propose a fix
"""
import asyncio
import json
import os
from datetime import timedelta

from django.core.management import BaseCommand

from assistant.bot import selfplay
from assistant.bot.domain import User
from assistant.bot.platforms.console import ConsolePlatform
from assistant.bot.session import BotSession
from assistant.bot.utils import get_bot_class
from assistant.conf import settings
from assistant.utils.sync import sync_to_async

DIALOGUES_FOLDER = "test_dialogs"


class Command(BaseCommand):
    help = "Self-play testing of a bot with LLM users and an LLM reviewer"

    def add_arguments(self, parser):
        parser.add_argument("command", choices=("run", "analyze"))
        parser.add_argument("bot_codename")
        parser.add_argument("-n", "--number", type=int, default=10)
        parser.add_argument("--tester-model", default=settings.get("TESTER_AI_MODEL", "gpt-4o-mini"))
        parser.add_argument("--analyzer-model", default=settings.get("ANALYZER_AI_MODEL", "gpt-4o"))
        parser.add_argument("--folder", default=DIALOGUES_FOLDER)

    def handle(self, *args, **o):
        asyncio.run(self.run(o) if o["command"] == "run" else self.analyze(o))

    async def run(self, o):
        from assistant.bot.management.commands.utils import get_instance
        from assistant.bot.services.dialog_service import get_dialog
        from assistant.bot.services.instance_service import InstanceLockAsync
        from assistant.bot.store import DjangoBotStore

        os.makedirs(o["folder"], exist_ok=True)
        bot_cls = get_bot_class(o["bot_codename"])
        for i in range(o["number"]):
            user = User(id="tester", username="ai_tester", first_name="AI", last_name="Tester", language_code="ru")
            instance = await sync_to_async(get_instance)(o["bot_codename"], "ai_platform", "tester", user)
            dialog = await sync_to_async(get_dialog)(instance, timedelta(days=1))
            session = BotSession(bot_cls, ConsolePlatform(printer=None), DjangoBotStore(), dialog, user=user,
                                 chat_id="tester", lock_factory=InstanceLockAsync)
            try:
                log = await selfplay.run_dialog(session, o["tester_model"])
            finally:
                await sync_to_async(dialog.delete)()
            path = os.path.join(o["folder"], f"dialog_{i + 1}.json")
            with open(path, "w", encoding="utf-8") as f:
                json.dump(log, f, ensure_ascii=False, indent=2)
            self.stdout.write(f"Dialog {i + 1} saved to {path}")

    async def analyze(self, o):
        files = sorted((f for f in os.listdir(o["folder"]) if f.startswith("dialog_") and f.endswith(".json")),
                       key=lambda x: int(x[7:-5]))
        results = []
        for name in files:
            with open(os.path.join(o["folder"], name), encoding="utf-8") as f:
                log = json.load(f)
            r = await selfplay.analyze_dialog(log, o["analyzer_model"])
            results.append({"dialog_file": name, **r})
        with open(os.path.join(o["folder"], "analysis_results.jsonl"), "w", encoding="utf-8") as w:
            for r in results:
                w.write(json.dumps(r, ensure_ascii=False) + "\n")
        self.stdout.write(self.style.NOTICE("Analysis results:"))
        for r in results:
            ok = not (r["warnings"] or r["errors"] or r["crashes"])
            self.stdout.write(f"\nDialog `{r['dialog_file']}`: " + (self.style.SUCCESS("OK") if ok else ""))
            for w in r["warnings"]:
                self.stdout.write(self.style.WARNING(f"- {w}"))
            for e in r["errors"]:
                self.stdout.write(self.style.ERROR(f"- {e}"))
            if r["crashes"]:
                self.stdout.write(self.style.NOTICE(f"- {r['crashes']} crashes"))
        proposal = await selfplay.summarize(results, o["analyzer_model"], len(files))
        if proposal:
            self.stdout.write(self.style.SUCCESS("\nProposed improvement:"))
            self.stdout.write(proposal)
        else:
            self.stdout.write(self.style.SUCCESS("\nNo deficiencies found."))
