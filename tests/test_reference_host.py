"""The reference's own host project against this library (``example/`` must run
unchanged).

The reference's ``example/`` (read-only at /root/reference/example) is loaded as it is -- nothing copied,
nothing patched:

  * ``example/bot/bot.py``: its ``TaskManagerBot`` (methods decorated in the class body with
    ``@AssistantBot.command``, ``command_start(self, *args, **kwargs)`` overriding the built-in) is
    imported straight from the reference file and driven through the in-memory bot session;
  * ``example/bot/admin.py`` registers Bot / Instance / Dialog / Message itself, so no library
    ``admin.py`` may register them (Django's autodiscover would raise ``AlreadyRegistered``); checked on
    the source, since Django is not importable here;
  * every ``assistant.*`` name the host imports, every ``assistant.*`` app it installs, its URL include
    and its beat task exist in this library.

Skipped where the reference tree is absent (e.g. the GPU box)."""
import ast
import asyncio
import importlib.util
import os

import pytest

REF = "/root/reference/example"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference host project not present")


def _load_reference_bot():
    spec = importlib.util.spec_from_file_location("reference_example_bot", os.path.join(REF, "bot", "bot.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture()
def session():
    from assistant.ai.providers.fake import FakeAIProvider
    from assistant.bot.platforms.api import CollectingPlatform
    from assistant.bot.session import BotSession

    FakeAIProvider.reset()
    mod = _load_reference_bot()
    yield BotSession.in_memory(mod.TaskManagerBot, CollectingPlatform(), codename="task_manager"), FakeAIProvider
    FakeAIProvider.reset()


def _send(s, text):
    return asyncio.run(s.send(text))


def _texts(answer):
    return [p.text for p in getattr(answer, "parts", [answer])]


def test_reference_task_manager_bot_runs_unchanged(session):
    s, fake = session
    start = _texts(_send(s, "/start"))
    assert start == ["🖖 Welcome to TaskBot!", "Choose action:"]  # the host's command_start override
    fake.script(["#create_task"])
    assert _send(s, "please add a task").text == "📝 Enter task name:"
    ans = _send(s, "Buy milk")
    assert ans.text == "Choose priority:" and ans.buttons[0][0].callback_data == "/priority high"
    assert _texts(_send(s, "/priority high")) == ["Selected priority: high", "Create task?\nBuy milk (high priority)"]
    assert _texts(_send(s, "/confirm_task"))[0] == "🎉 Task created!"
    assert "1. Buy milk ❗" in _send(s, "/list").text
    assert s.dialog.instance.state["tasks"] == [{"title": "Buy milk", "priority": "high"}]
    assert _send(s, "/new_task").text == "📝 Enter task name:"
    assert _send(s, "/cancel").text == "❌ Operation cancelled"
    assert not s.dialog.instance.state.get("awaiting_input")
    assert _send(s, "/help").text.startswith("🤖 *TaskBot - Task Management*")
    fake.script(["#list_tasks"])
    assert _send(s, "what do I have to do").text.startswith("📋 Task list:")
    fake.script(["#other", "Sure, here you go."])
    assert _send(s, "what is the weather").text == "🤖 Sure, here you go."
    assert not fake._script


def test_reference_commands_stay_in_the_host_class(session):
    """In-class ``@AssistantBot.command`` methods belong to the host's subclass: the base bot (and any
    other bot class) does not answer them."""
    from assistant.bot.assistant_bot import AssistantBot
    from assistant.bot.platforms.api import CollectingPlatform
    from assistant.bot.session import BotSession

    s, _ = session
    host_patterns = {p.pattern for p, _ in s.bot_cls._command_handlers}
    assert {"/priority (high|medium|low)", "/confirm_task", "/cancel", "/list", "/new_task"} <= host_patterns
    assert not any(p.pattern in host_patterns for p, _ in AssistantBot._command_handlers)
    base = BotSession.in_memory(AssistantBot, CollectingPlatform())
    assert _send(base, "/new_task").text == "`Unknown command.`"


def _registered_models(path):
    """Model names registered by an admin module: ``admin.site.register(M, ...)`` calls (also over a
    tuple loop) and ``@admin.register(M, ...)`` decorators."""
    tree = ast.parse(open(path, encoding="utf-8").read())
    names = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute) and node.func.attr == "register":
            for a in node.args[:1]:
                if isinstance(a, ast.Name):
                    names.add(a.id)
    return names


def test_no_library_admin_registers_a_host_model():
    host = _registered_models(os.path.join(REF, "bot", "admin.py"))
    assert host == {"Bot", "Instance", "Dialog", "Message"}
    offenders = {}
    for root, _, files in os.walk(os.path.join(REPO, "assistant")):
        for f in files:
            if f == "admin.py":
                got = _registered_models(os.path.join(root, f))
                if got:
                    offenders[os.path.relpath(os.path.join(root, f), REPO)] = sorted(got)
    # the reference library registers nothing itself (its @admin.register lines are commented out)
    assert offenders == {}


def _defined_names(module):
    path = os.path.join(REPO, *module.split("."))
    path = os.path.join(path, "__init__.py") if os.path.isdir(path) else path + ".py"
    tree = ast.parse(open(path, encoding="utf-8").read())
    names = set()
    for node in ast.walk(tree):
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            names.add(node.name)
        elif isinstance(node, ast.Assign):
            names |= {t.id for t in node.targets if isinstance(t, ast.Name)}
        elif isinstance(node, ast.AnnAssign) and isinstance(node.target, ast.Name):
            names.add(node.target.id)
        elif isinstance(node, (ast.Import, ast.ImportFrom)):
            names |= {(a.asname or a.name).split(".")[0] for a in node.names}
    return names


def test_every_library_name_the_host_imports_exists():
    missing = []
    for root, _, files in os.walk(REF):
        for f in files:
            if not f.endswith(".py"):
                continue
            tree = ast.parse(open(os.path.join(root, f), encoding="utf-8").read())
            for node in ast.walk(tree):
                if isinstance(node, ast.ImportFrom) and (node.module or "").startswith("assistant"):
                    have = _defined_names(node.module)
                    missing += [f"{node.module}.{a.name}" for a in node.names if a.name not in have]
                elif isinstance(node, ast.Import):
                    for a in node.names:
                        if a.name.startswith("assistant"):
                            p = os.path.join(REPO, *a.name.split("."))
                            if not (os.path.isdir(p) or os.path.exists(p + ".py")):
                                missing.append(a.name)
    assert missing == []


def test_host_settings_urls_and_beat_task_resolve():
    tree = ast.parse(open(os.path.join(REF, "example", "settings.py"), encoding="utf-8").read())
    apps, bots, beat = [], {}, []
    for node in ast.walk(tree):
        if isinstance(node, ast.Assign) and isinstance(node.targets[0], ast.Name):
            name = node.targets[0].id
            if name == "INSTALLED_APPS":
                apps = [e.value for e in node.value.elts]
            elif name == "BOTS":
                bots = {k.value: {kk.value: vv for kk, vv in zip(v.keys, v.values)}
                        for k, v in zip(node.value.keys, node.value.values)}
            elif name == "CELERY_BEAT_SCHEDULE":
                beat = [v.values[[k.value for k in v.keys].index("task")].value for v in node.value.values]
    lib_apps = [a for a in apps if a.startswith("assistant.")]
    assert lib_apps and all(os.path.exists(os.path.join(REPO, *a.split("."), "apps.py")) for a in lib_apps)
    # the host's bot class path resolves inside the repo's example/ (same layout)
    cls_path = bots["task_manager"]["class"].value
    mod, cls = cls_path.rsplit(".", 1)
    assert cls in _defined_names_in(os.path.join(REPO, "example", *mod.split(".")) + ".py")
    urls = open(os.path.join(REF, "example", "urls.py"), encoding="utf-8").read()
    assert "include('assistant.assistant.urls')" in urls
    assert os.path.exists(os.path.join(REPO, "assistant", "assistant", "urls.py"))
    tasks_src = open(os.path.join(REPO, "assistant", "broadcasting", "tasks.py"), encoding="utf-8").read()
    assert beat and all(f'name="{t}"' in tasks_src for t in beat)


def _defined_names_in(path):
    return {n.name for n in ast.walk(ast.parse(open(path, encoding="utf-8").read())) if isinstance(n, ast.ClassDef)}


def test_repo_example_registers_what_the_reference_host_registers():
    assert _registered_models(os.path.join(REPO, "example", "bot", "admin.py")) == \
        _registered_models(os.path.join(REF, "bot", "admin.py"))
