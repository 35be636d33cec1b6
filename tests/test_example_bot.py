"""The example TaskManagerBot end to end on the in-memory store (reference example/bot/bot.py):
intent routing, the title -> priority -> confirm state machine through callback commands, cancel,
listing, and the overridden /start and /help."""
import asyncio
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "example"))

from assistant.ai.providers.fake import FakeAIProvider  # noqa: E402
from assistant.bot.assistant_bot import AssistantBot  # noqa: E402
from assistant.bot.platforms.api import CollectingPlatform  # noqa: E402
from assistant.bot.session import BotSession  # noqa: E402
from bot.bot import TaskManagerBot  # noqa: E402


@pytest.fixture(autouse=True)
def _fake():
    FakeAIProvider.reset()
    yield
    FakeAIProvider.reset()


def send(s, text):
    return asyncio.run(s.send(text))


def texts(answer):
    return [p.text for p in getattr(answer, "parts", [answer])]


def test_task_flow():
    s = BotSession.in_memory(TaskManagerBot, CollectingPlatform(), codename="task_manager")
    assert texts(send(s, "/start"))[0].startswith("🖖 Welcome")
    FakeAIProvider.script(["#create_task"])
    assert send(s, "I need to add a task").text == "📝 Enter task name:"
    ans = send(s, "Buy milk")
    assert ans.text == "Choose priority:" and ans.buttons[0][0].callback_data == "/priority high"
    ans = send(s, "/priority high")
    assert texts(ans) == ["Selected priority: high", "Create task?\nBuy milk (high priority)"]
    assert texts(send(s, "/confirm_task"))[0] == "🎉 Task created!"
    assert "1. Buy milk ❗" in send(s, "/list").text
    FakeAIProvider.script(["#list_tasks"])
    assert "Buy milk" in send(s, "show me my tasks").text
    FakeAIProvider.script(["#other", "Sure, here you go."])
    assert send(s, "what's the weather").text == "🤖 Sure, here you go."
    assert not FakeAIProvider._script


def test_cancel_keeps_tasks_and_help_override():
    s = BotSession.in_memory(TaskManagerBot, CollectingPlatform(), codename="task_manager")
    s.dialog.instance.state["tasks"] = [{"title": "old", "priority": "low"}]
    assert send(s, "/new_task").text == "📝 Enter task name:"
    assert send(s, "/cancel").text == "❌ Operation cancelled"
    assert s.dialog.instance.state["tasks"] == [{"title": "old", "priority": "low"}]
    assert not s.dialog.instance.state.get("awaiting_input")
    assert send(s, "/help").text.startswith("🤖 *TaskBot")
    assert send(s, "/priority low").text == "Nothing to set a priority for."


def test_commands_do_not_leak_into_base_bot():
    s = BotSession.in_memory(AssistantBot, CollectingPlatform())
    assert send(s, "/list").text == "`Unknown command.`"
