"""Task-manager demo bot (reference example/bot/bot.py:17-359).

Shows the extension points of ``AssistantBot``:
  * ``get_answer_to_messages`` replaced by intent routing (fast-model classification into
    #create_task / #list_tasks / #other) instead of the RAG pipeline;
  * a small state machine kept in ``instance.state`` (title -> priority -> confirmation);
  * ``@AssistantBot.command`` handlers written as methods of the class, as the reference host does
    (the library moves them into this class's own registry), including ``command_start`` /
    ``command_help``, which replace the built-in /start and /help.

Tasks live in the instance state (``state['tasks']``), so the demo needs no models of its own.
"""
from __future__ import annotations

import logging
import re
from typing import Optional

from assistant.ai.providers.base import AIDebugger
from assistant.bot.assistant_bot import AssistantBot
from assistant.bot.domain import Answer, Button, MultiPartAnswer, SingleAnswer
from assistant.bot.services.context_service.utils import add_system_message
from assistant.utils.repeat_until import repeat_until

logger = logging.getLogger(__name__)

INTENTS = ("#create_task", "#list_tasks", "#other")
PRIORITY_ICON = {"high": "❗", "medium": "🔰", "low": "🐌"}
MAIN_MENU = [[Button("➕ New task", callback_data="/new_task")], [Button("📋 My tasks", callback_data="/list")],
             [Button("❓ Help", callback_data="/help")]]


def pick_intent(text: str) -> str:
    for tag in INTENTS:
        if tag in (text or ""):
            return tag
    return "#other"


class TaskManagerBot(AssistantBot):
    """Creates and lists tasks kept in the instance state."""

    # -------------------------------------------------------------------------------- routing
    async def get_answer_to_messages(self, messages, debug_info, do_interrupt) -> Answer:
        if self.instance.state.get("awaiting_input"):
            return await self.handle_state_input(messages)
        intent = await self.classify_intent(messages, debug_info)
        if intent == "#create_task":
            return await self.initiate_task_creation()
        if intent == "#list_tasks":
            return self.task_list()
        return await self.general_answer(messages, debug_info)

    async def classify_intent(self, messages, debug_info) -> str:
        instruction = ("Classify the user's last request:\n"
                       "#create_task - they want to create a new task\n"
                       "#list_tasks - they want to see their tasks\n"
                       "#other - anything else\n"
                       "Answer with the tag only.")
        with AIDebugger(self._fast_ai, debug_info, "intent_classification") as dbg:
            resp = await repeat_until(dbg.ai.get_response, add_system_message(messages, instruction),
                                      max_tokens=16, condition=lambda r: any(t in str(r.result) for t in INTENTS))
            intent = pick_intent(str(resp.result))
            dbg.info["detected_intent"] = intent
        return intent

    async def general_answer(self, messages, debug_info) -> SingleAnswer:
        with AIDebugger(self._strong_ai, debug_info, "general_response") as dbg:
            resp = await repeat_until(dbg.ai.get_response, messages, max_attempts=3,
                                      condition=lambda r: len(str(r.result)) < 500)
        return SingleAnswer(f"🤖 {resp.result}")

    # -------------------------------------------------------------------------- state machine
    async def initiate_task_creation(self) -> SingleAnswer:
        await self.update_state({"awaiting_input": "task_title", "new_task": {}})
        return SingleAnswer("📝 Enter task name:", buttons=[[Button("Cancel", callback_data="/cancel")]])

    async def handle_state_input(self, messages) -> SingleAnswer:
        if self.instance.state.get("awaiting_input") == "task_title":
            title = (messages[-1]["content"] or "").strip()
            await self.update_state({"awaiting_input": "task_priority", "new_task": {"title": title}})
            return SingleAnswer("Choose priority:", buttons=[
                [Button("❗High", callback_data="/priority high")],
                [Button("🔰 Medium", callback_data="/priority medium")],
                [Button("🐌 Low", callback_data="/priority low")]])
        return SingleAnswer("Please use the buttons above, or /cancel.", no_store=True)

    def task_list(self) -> SingleAnswer:
        tasks = self.instance.state.get("tasks") or []
        if tasks:
            body = "\n".join(f"{i}. {t['title']} {PRIORITY_ICON.get(t.get('priority'), '')}".rstrip()
                             for i, t in enumerate(tasks, 1))
        else:
            body = "The task list is empty."
        return SingleAnswer(f"📋 Task list:\n\n{body}", buttons=[
            [Button("➕ New task", callback_data="/new_task")], [Button("🏠 Main menu", callback_data="/start")]])

    # ------------------------------------------------------------------------------- commands
    @AssistantBot.command(r"/priority (high|medium|low)$")
    async def set_priority(self, match: re.Match, message_id: Optional[int] = None) -> Answer:
        if self.instance.state.get("awaiting_input") != "task_priority":
            return SingleAnswer("Nothing to set a priority for.", no_store=True)
        task = dict(self.instance.state.get("new_task") or {}, priority=match.group(1))
        await self.update_state({"awaiting_input": "confirming", "new_task": task})
        return MultiPartAnswer([
            SingleAnswer(f"Selected priority: {task['priority']}"),
            SingleAnswer(f"Create task?\n{task['title']} ({task['priority']} priority)", buttons=[
                [Button("✅ Confirm", callback_data="/confirm_task")],
                [Button("❌ Cancel", callback_data="/cancel")]]),
        ])

    @AssistantBot.command(r"/confirm_task$")
    async def confirm_task(self, match=None, message_id=None) -> Answer:
        if self.instance.state.get("awaiting_input") != "confirming":
            return SingleAnswer("Nothing to confirm.", no_store=True)
        tasks = list(self.instance.state.get("tasks") or []) + [self.instance.state["new_task"]]
        logger.info("task created: %s", tasks[-1])
        await self.update_state({"tasks": tasks, "awaiting_input": None, "new_task": None})
        return MultiPartAnswer([SingleAnswer("🎉 Task created!"), SingleAnswer("What's next?", buttons=[
            [Button("➕ New task", callback_data="/new_task")], [Button("📋 Task list", callback_data="/list")]])])

    @AssistantBot.command(r"/cancel$")
    async def cancel(self, match=None, message_id=None) -> Answer:
        tasks = self.instance.state.get("tasks") or []
        await self.clear_state()
        await self.update_state({"tasks": tasks})  # keep the task list, drop the pending operation
        return SingleAnswer("❌ Operation cancelled", buttons=[[Button("Main menu", callback_data="/start")]])

    @AssistantBot.command(r"/list$")
    async def list_tasks(self, match=None, message_id=None) -> Answer:
        return self.task_list()

    @AssistantBot.command(r"/new_task$")
    async def new_task(self, match=None, message_id=None) -> Answer:
        return await self.initiate_task_creation()

    @AssistantBot.command(r"/start")
    async def command_start(self, *args, **kwargs) -> Answer:
        return MultiPartAnswer([SingleAnswer("🖖 Welcome to TaskBot!"),
                                SingleAnswer("Choose action:", buttons=MAIN_MENU)])

    @AssistantBot.command(r"/help")
    async def command_help(self, *args, **kwargs) -> Answer:
        return SingleAnswer("🤖 *TaskBot - Task Management*\n\n📝 *Commands:*\n\n"
                            "• /new_task - Create a task\n• /list - Task list\n• /cancel - Cancel operation\n"
                            "• /start - Main menu",
                            buttons=[[Button("🏠 Main menu", callback_data="/start")],
                                     [Button("➕ New task", callback_data="/new_task")]])
