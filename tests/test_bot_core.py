"""Conversation layer without Django: MarkdownV2 formatting, the Telegram platform over a fake Bot API
transport, and full update -> answer flows of ``AssistantBot`` on the in-memory store with the
in-memory knowledge base (engine VectorIndex on CPU) and the deterministic fake AI providers.

Behaviour specs follow the reference's intent (tests/bot_tests/test_assistant_bot.py:17-108: a fake
platform receives exactly one answer; the AI is faked at the provider boundary)."""
import asyncio

import pytest

from assistant.ai.domain import AIResponse
from assistant.ai.providers.fake import FakeAIProvider, FakeEmbedder
from assistant.bot.assistant_bot import AssistantBot, merge_role_runs, parse_whitelist, split_thinking
from assistant.bot.domain import Audio, Button, SingleAnswer
from assistant.bot.exceptions import UserUnavailableError
from assistant.bot.platforms.api import CollectingPlatform
from assistant.bot.platforms.telegram.format import (TelegramMarkdownV2FormattedText, escape_markdownV2,
                                                     format_markdownV2)
from assistant.bot.platforms.telegram.platform import TelegramAPI, TelegramBotPlatform
from assistant.bot.session import BotSession
from assistant.rag.knowledge import KnowledgeDocument, MemoryKnowledgeBase, WikiRef


def run(coro):
    return asyncio.run(coro)


@pytest.fixture(autouse=True)
def _reset_fake():
    FakeAIProvider.reset()
    yield
    FakeAIProvider.reset()


# ------------------------------------------------------------------------------------- formatting

@pytest.mark.parametrize("src,expected", [
    ("plain text.", "plain text\\."),
    ("**bold** and *it*", "*bold* and _it_"),
    ("__bold__ _it_", "*bold* _it_"),
    ("~~gone~~", "~gone~"),
    ("use `a_b(c)`", "use `a_b(c)`"),
    ("[site](http://x.org/a_b)", "[site](http://x.org/a_b)"),
    ("# Head (1)", "*Head \\(1\\)*"),
    ("a = b + c!", "a \\= b \\+ c\\!"),
    ("snake_case_word", "snake\\_case\\_word"),
])
def test_inline_and_headings(src, expected):
    assert format_markdownV2(src) == expected


def test_blocks_lists_code_quote():
    src = "Intro:\n\n- one\n  - nested.\n- two\n\n1. first\n2. second\n\n```py\nx = `1`\\n\n```\n\n> said"
    out = format_markdownV2(src)
    assert out.split("\n\n") == [
        "Intro:",
        "\\- one\n  \\- nested\\.\n\\- two",
        "1\\. first\n2\\. second",
        "```\nx = \\`1\\`\\\\n\n```",
        ">said",
    ]


def test_formatted_text_keeps_raw():
    t = TelegramMarkdownV2FormattedText("**x**.")
    assert str(t) == "*x*\\." and t.raw_text == "**x**."
    assert escape_markdownV2("a.b") == "a\\.b"


# ------------------------------------------------------------------------------------- telegram

class FakeTransport:
    def __init__(self, responses=None):
        self.calls = []
        self.responses = dict(responses or {})

    async def __call__(self, method, params, files):
        self.calls.append((method, params, files))
        r = self.responses.get(method)
        if isinstance(r, list):
            r = r.pop(0)
        if callable(r):
            r = r(params)
        if method == "__download__":
            return 200, b"\x89PNGdata"
        return (200, {"ok": True, "result": r}) if r is None or not isinstance(r, tuple) else r


def test_telegram_update_conversion():
    tr = FakeTransport({"getFile": {"file_path": "photos/file_1.jpg"}})
    platform = TelegramBotPlatform("T", api=TelegramAPI("T", transport=tr))
    msg = {"update_id": 1, "message": {
        "message_id": 7, "chat": {"id": 42}, "from": {"id": 42, "username": "u", "language_code": "en"},
        "caption": "look", "photo": [{"file_id": "s", "file_unique_id": "su"}, {"file_id": "b", "file_unique_id": "bu"}],
        "contact": {"phone_number": "+100"}}}
    upd = run(platform.get_update(msg))
    assert (upd.chat_id, upd.message_id, upd.text, upd.phone_number) == ("42", 7, "look", "+100")
    assert upd.photo.file_id == "bu" and upd.photo.extension == "jpg" and upd.photo.content == b"\x89PNGdata"
    assert tr.calls[0][:2] == ("getFile", {"file_id": "b"})
    cb = {"callback_query": {"id": "c", "from": {"id": 5}, "message": {"message_id": 9}, "data": "/continue"}}
    upd = run(platform.get_update(cb))
    assert (upd.chat_id, upd.message_id, upd.text, upd.user.id) == ("5", 9, "/continue", "5")


def test_telegram_post_answer_markup_and_fallback():
    bad = (400, {"ok": False, "error_code": 400, "description": "Bad Request: can't parse entities"})
    tr = FakeTransport({"sendMessage": [bad, None]})
    platform = TelegramBotPlatform("T", api=TelegramAPI("T", transport=tr))
    ans = SingleAnswer("**hi**.", buttons=[[Button("Go", callback_data="/go"), Button("Site", url="http://x")]])
    run(platform.post_answer("1", ans))
    (m1, p1, _), (m2, p2, _) = tr.calls
    assert m1 == m2 == "sendMessage"
    assert p1["parse_mode"] == "MarkdownV2" and p1["text"] == "*hi*\\."
    assert "parse_mode" not in p2 and p2["text"] == "**hi**."
    assert p1["reply_markup"] == {"inline_keyboard": [[{"text": "Go", "callback_data": "/go"},
                                                       {"text": "Site", "url": "http://x"}]]}
    tr2 = FakeTransport()
    platform2 = TelegramBotPlatform("T", api=TelegramAPI("T", transport=tr2))
    run(platform2.post_answer("1", SingleAnswer("x", reply_keyboard=[[Button("Share", request_contact=True)]],
                                                audio=Audio(b"ID3", "a.mp3"))))
    assert [c[0] for c in tr2.calls] == ["sendAudio", "sendMessage"]
    assert tr2.calls[0][2]["audio"] == ("a.mp3", b"ID3")
    kb = tr2.calls[1][1]["reply_markup"]
    assert kb["one_time_keyboard"] and kb["keyboard"][0][0]["request_contact"]
    tr3 = FakeTransport()
    run(TelegramBotPlatform("T", api=TelegramAPI("T", transport=tr3)).post_answer("1", SingleAnswer("x")))
    assert tr3.calls[0][1]["reply_markup"] == {"remove_keyboard": True}


def test_telegram_forbidden():
    blocked = (403, {"ok": False, "error_code": 403, "description": "Forbidden: bot was blocked by the user"})
    kicked = (403, {"ok": False, "error_code": 403, "description": "Forbidden: bot was kicked from the group chat"})
    p = TelegramBotPlatform("T", api=TelegramAPI("T", transport=FakeTransport({"sendMessage": [blocked]})))
    with pytest.raises(UserUnavailableError) as e:
        run(p.post_answer("77", SingleAnswer("x")))
    assert e.value.chat_id == "77"
    p = TelegramBotPlatform("T", api=TelegramAPI("T", transport=FakeTransport({"sendMessage": [kicked]})))
    run(p.post_answer("77", SingleAnswer("x")))  # logged, not raised


# ------------------------------------------------------------------------------------- bot logic

def test_helpers():
    thinking, text = split_thinking("<think> plan </think>Answer")
    assert thinking == "plan" and text == "Answer"
    msgs = [{"role": "system", "content": "s"}, {"role": "user", "content": "/start"},
            {"role": "user", "content": "a"}, {"role": "user", "content": "b"}, {"role": "assistant", "content": "c"}]
    assert merge_role_runs(msgs) == [{"role": "system", "content": "s"}, {"role": "user", "content": "a\nb"},
                                     {"role": "assistant", "content": "c"}]
    assert parse_whitelist("@alice\n 123 \n\n") == {"alice", "123"}


def _session(**kw):
    return BotSession.in_memory(AssistantBot, CollectingPlatform(), system_text="You are a helpful bot.", **kw)


def test_commands():
    s = _session(start_text="Welcome!", help_text="Help text")
    assert run(s.send("/start")).text == "Welcome!"
    assert run(s.send("/help")).text == "Help text"
    assert run(s.send("/nonsense")).text == "`Unknown command.`"
    assert run(s.send("/model fake:strong")).text.startswith("`Model`")
    assert s.dialog.instance.state["model"] == "fake:strong"
    assert "fake:strong" in run(s.send("/model")).text
    models = run(s.send("/models"))
    assert models.buttons and models.buttons[0][0].callback_data.startswith("/model ")
    assert run(s.send("/debug")).text.startswith("```json")
    old = s.dialog
    assert run(s.send("/new")).text == "`New dialog started.`" and old.is_completed
    assert [c for c, _ in s.platform.sent] == [s.chat_id] * 8
    # commands are never stored as dialog messages on the bot side
    assert all(m.role == "user" for m in s.store.messages(old))


def test_custom_command_registry_is_per_class():
    class MyBot(AssistantBot):
        pass

    @MyBot.command(r"/ping (\w+)")
    async def ping(bot, match, message_id):
        return SingleAnswer(f"pong {match.group(1)}", no_store=True)

    s = BotSession.in_memory(MyBot, CollectingPlatform())
    assert run(s.send("/ping x")).text == "pong x"
    s2 = _session()
    assert run(s2.send("/ping x")).text == "`Unknown command.`"


def test_whitelist():
    s = _session()
    s.dialog.instance.bot.is_whitelist_enabled = True
    s.dialog.instance.bot.telegram_whitelist = "@someone"
    assert run(s.send("hello")).text == "`Authorization required.`"
    s.dialog.instance.bot.telegram_whitelist = "@someone\ntester"
    FakeAIProvider.script(["hi there"])
    assert run(s.send("hello")).text == "hi there"


def _kb():
    emb = FakeEmbedder()
    kb = MemoryKnowledgeBase(emb.embeddings, dim=emb.dim if hasattr(emb, "dim") else 768, device="cpu")
    docs = [
        (KnowledgeDocument(1, "Shipping", "We ship worldwide in 5 days.", WikiRef("Store / Shipping", 10)),
         ["how long does shipping take", "do you ship worldwide", "shipping time delivery days",
          "where do you deliver", "delivery speed of orders"], "Store"),
        (KnowledgeDocument(2, "Returns", "Returns are accepted within 30 days.", WikiRef("Store / Returns", 11)),
         ["can i return an item", "return policy days", "how to send back a product", "refund for returns",
          "returning goods rules"], "Store"),
    ]
    for doc, qs, topic in docs:
        run(kb.add_document(doc, qs, topic))
    return kb


def test_rag_dialog_answer_uses_retrieved_document():
    s = _session()
    s.dialog.instance.bot.knowledge = _kb()
    FakeAIProvider.script([{"topic": "Store"}, {"question": None}, "It takes <b>5</b> days."])
    ans = run(s.send("how long does shipping delivery take"))
    assert ans.text == "It takes <b>5</b> days." and not ans.no_store
    final = FakeAIProvider.requests[-1]["messages"]
    assert "We ship worldwide in 5 days." in final[-1]["content"]
    assert "Store / Shipping" in final[-1]["content"]
    dialog_msgs = s.store.messages(s.dialog)
    assert [m.role for m in dialog_msgs] == ["user", "assistant"]
    assert len(s.platform.sent) == 1


def test_same_question_shortcut_and_small_talk():
    s = _session()
    s.dialog.instance.bot.knowledge = _kb()
    FakeAIProvider.script([{"topic": "Store"}, {"question": 1}, "30 days"])
    assert run(s.send("return policy days")).text == "30 days"
    final = FakeAIProvider.requests[-1]["messages"][-1]["content"]
    assert "Returns are accepted within 30 days." in final
    FakeAIProvider.reset()
    FakeAIProvider.script([{"topic": "Small talk"}, "Hello!"])
    assert run(s.send("hi")).text == "Hello!"
    # small talk skips retrieval: the final prompt has no document
    assert "Returns are accepted" not in FakeAIProvider.requests[-1]["messages"][-1]["content"]


def test_thinking_tags_and_continue_button():
    s = _session()
    FakeAIProvider.script([AIResponse("<think>reasoning</think>#text\nVisible part", {"model": "x"}, True)])
    ans = run(s.send("tell me"))
    assert ans.thinking == "reasoning"
    assert ans.text == "Visible part"
    assert ans.buttons[0][0].callback_data == "/continue"
    assert ans.raw_text.startswith("<think>")


def test_no_double_answer_when_already_answered():
    s = _session()
    FakeAIProvider.script(["first"])
    assert run(s.send("q1")).text == "first"
    # a duplicate delivery of the same update must not produce a second answer
    bot = AssistantBot(dialog=s.dialog, platform=s.platform, store=s.store)
    from assistant.bot.domain import Update
    assert run(bot.handle_update(Update(chat_id=s.chat_id, message_id=s.message_id, text="q1"))) is None


def test_unavailable_user_is_marked():
    class Refusing(CollectingPlatform):
        async def post_answer(self, chat_id, answer):
            raise UserUnavailableError(chat_id)

    s = BotSession.in_memory(AssistantBot, Refusing(), start_text="hi")
    run(s.send("/start"))
    assert s.dialog.instance.is_unavailable
    FakeAIProvider.script(["ok"])
    run(s.send("hello again"))  # writing again clears the flag before answering
    assert s.dialog.instance.is_unavailable  # ...and the refused delivery sets it again


def test_selfplay_dialog_and_analysis():
    from assistant.bot import selfplay
    from assistant.bot.platforms.console import ConsolePlatform

    s = BotSession.in_memory(AssistantBot, ConsolePlatform(printer=None), start_text="Hi! Ask me.")
    # tester: /start, q1, q2 ; bot answers q1, q2 ; control says end after turn 3
    FakeAIProvider.script(["/start", "what is this?", "bot answer 1", "thanks, bye", "bot answer 2", "end"])
    log = asyncio.run(selfplay.run_dialog(s, "test", max_turns=5, persona="- language: english"))
    assert [e["role"] for e in log] == ["user", "assistant"] * 3
    assert log[1]["text"] == "Hi! Ask me." and log[3]["text"] == "bot answer 1"
    FakeAIProvider.script([{"warnings": ["w1"], "errors": []}])
    r = asyncio.run(selfplay.analyze_dialog(log, "test"))
    assert r == {"warnings": ["w1"], "errors": [], "crashes": 0}
    FakeAIProvider.script(["Fix the greeting."])
    assert asyncio.run(selfplay.summarize([r], "test", 1)) == "Fix the greeting."
    assert asyncio.run(selfplay.summarize([{"warnings": [], "errors": [], "crashes": 0}], "test", 1)) is None
