"""LLM self-play QA harness (reference bot/management/commands/tester.py:37-453), Django-free.

``run_dialog``: a tester LLM role-plays a user with a random persona against any bot session until it
says goodbye (decided by a control LLM after turn 2) or ``max_turns``.  ``analyze_dialog`` asks an
analyzer LLM for JSON ``{"warnings": [...], "errors": [...]}``; ``summarize`` counts them plus crashes
(answers containing the error phrase) and asks for the single highest-priority improvement.
"""
from __future__ import annotations

import itertools
import random
from typing import Dict, List, Optional

from assistant.ai.dialog import AIDialog
from assistant.ai.domain import Message, system_message
from assistant.utils.repeat_until import repeat_until

PERSONA_TRAITS = {
    "age group": ["teenager", "young adult", "middle-aged", "elderly"],
    "knowledge level": ["beginner", "intermediate", "expert"],
    "message length": ["very short", "short", "detailed"],
    "tone": ["formal", "casual", "humorous", "blunt"],
    "interest": ["very interested", "curious but reserved", "barely interested"],
    "attitude to advice": ["open-minded", "skeptical", "resistant"],
    "mood": ["cheerful", "thoughtful", "impatient", "nervous"],
    "question style": ["asks many follow-ups", "asks one thing and leaves", "wanders between topics"],
    "vocabulary": ["technical terms", "plain words", "slang"],
}


def random_persona(rng: random.Random = None, language: str = "russian") -> str:
    rng = rng or random
    traits = {"language": language, **{k: rng.choice(v) for k, v in PERSONA_TRAITS.items()}}
    return "\n".join(f"- {k}: {v}" for k, v in traits.items())


def tester_prompt(persona: str) -> str:
    return ("Play the role of a person chatting with a bot. Write only your next message.\n"
            f"Your persona:\n{persona}\n"
            "Invent any other details about yourself that fit the conversation.\n"
            "Your very first message is exactly \"/start\"; never send it again afterwards.\n"
            "When the conversation has reached a natural end you may say goodbye.")


async def run_dialog(session, tester_model: str, max_turns: int = 10, persona: Optional[str] = None,
                     rng: random.Random = None) -> List[Dict]:
    """Drive ``session`` (a ``BotSession``) with an LLM user; returns the dialog log."""
    log: List[Dict] = []
    user_ai, control_ai = AIDialog(tester_model), AIDialog(tester_model)
    prompt = system_message(tester_prompt(persona or random_persona(rng)))
    for turn in range(1, max_turns + 1):
        # roles are mirrored: to the tester LLM the bot is the "user"
        history: List[Message] = [Message(role="user" if e["role"] == "assistant" else "assistant",
                                          content=e["text"] or "") for e in log]
        text = (await user_ai.get_response([prompt] + history, max_tokens=150)).result.strip()
        log.append({"role": "user", "text": text})
        answer = await session.send(text)
        parts = getattr(answer, "parts", None) or ([answer] if answer else [])
        for part in parts:
            entry = {"role": "assistant", "text": part.text}
            if part.buttons:
                entry["buttons"] = [[{"text": b.text, "callback_data": b.callback_data, "url": b.url} for b in row]
                                    for row in part.buttons]
            log.append(entry)
        if turn > 2:
            decision = await repeat_until(
                control_ai.get_response,
                history + [system_message("Given the dialog so far, will the user continue or end it? "
                                          "Reply with one word: continue or end.")],
                max_tokens=10, condition=lambda r: str(r.result).strip().lower() in ("continue", "end"))
            if str(decision.result).strip().lower() != "continue":
                break
    return log


def _dialog_text(log: List[Dict]) -> str:
    return "".join(f"{'User' if e['role'] == 'user' else 'Bot'}: {e.get('text')}\n" for e in log)


def analysis_prompt(dialog_text: str, language: str = "Russian") -> str:
    return ("You review chatbot conversations for quality.\n"
            "Find what the bot should improve in the conversation below, looking at: language problems "
            "(grammar, punctuation, broken formatting); misunderstood questions, irrelevant or wrong "
            "information; unnatural, rude or mismatched tone; missed chances to suggest a helpful next step.\n"
            "Split findings into `warnings` (minor) and `errors` (serious); leave a list empty when nothing "
            f"applies. Write each finding in {language}, quoting the dialog where possible.\n"
            "`/start` is the technical first message of a new user.\n"
            f"Conversation:\n{dialog_text}\n"
            "Reply with JSON exactly like:\n```json\n{\n  \"warnings\": [\"...\"],\n  \"errors\": [\"...\"]\n}\n```")


def _valid_analysis(r) -> bool:
    return isinstance(r.result, dict) and all(isinstance(r.result.get(k), (list, type(None)))
                                              for k in ("warnings", "errors"))


async def analyze_dialog(log: List[Dict], analyzer_model: str, crash_marker: str = "An error occurred ") -> Dict:
    text = _dialog_text(log)
    resp = await repeat_until(AIDialog(analyzer_model).get_response, [system_message(analysis_prompt(text))],
                              max_tokens=1024, json_format=True, condition=_valid_analysis)
    return {"warnings": resp.result.get("warnings") or [], "errors": resp.result.get("errors") or [],
            "crashes": text.count(crash_marker)}


async def summarize(results: List[Dict], analyzer_model: str, n_dialogs: int) -> Optional[str]:
    warnings = list(itertools.chain(*(r["warnings"] for r in results)))
    errors = list(itertools.chain(*(r["errors"] for r in results)))
    crashes = sum(r["crashes"] for r in results)
    if not (warnings or errors or crashes):
        return None
    prompt = (f"Below are problems found in {n_dialogs} conversations between users and a bot.\n"
              "Propose the ONE improvement to do first, weighing how many users it affects, how much it helps, "
              "how sure we are and how much work it is. Describe it in detail, in Russian, without naming a "
              "scoring framework.\n"
              "Warnings:\n" + "\n".join(f"- \"{w}\"" for w in warnings) + "\n"
              "Errors:\n" + "\n".join(f"- \"{e}\"" for e in errors) + "\n")
    if crashes:
        prompt += f"The bot crashed {crashes} times while answering; crashes come first.\n"
    return (await AIDialog(analyzer_model).get_response([system_message(prompt)], max_tokens=500)).result.strip()
