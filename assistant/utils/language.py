"""Language identification restricted to English / Russian (reference utils/language.py used
``langid.set_languages(['en', 'ru'])``).  langid is not a dependency here: a script + stop-word +
character-bigram scorer decides between the two languages, which is the only decision the pipeline
makes with it (the 'ru' checks of the ingest steps)."""
from __future__ import annotations

import logging
import re

logger = logging.getLogger(__name__)

LANGUAGES = ("en", "ru")

_EN_STOP = set("the a an and or of to in is are was were be been it this that for on with as by at from not "
               "you your i we they he she do does did have has had what which who how why when where can will "
               "would should could there their my me our us if but so no yes".split())
_RU_STOP = set("и в во не что он на я с со как а то все она так его но да ты к у же вы за бы по только ее мне "
               "было вот от меня еще нет о из ему теперь когда даже ну вдруг ли если уже или ни быть был него до "
               "вас нибудь опять уж вам ведь там потом себя ничего ей может они тут где есть надо ней для мы тебя "
               "их чем была сам чтоб без будто чего раз тоже себе под будет ж тогда кто этот того потому этого "
               "какой совсем ним здесь этом один почти мой тем чтобы нее сейчас были куда зачем всех никогда "
               "можно при наконец два об другой хоть после над больше тот через эти нас про всего них какая много "
               "разве три эту моя впрочем хорошо свою этой перед иногда лучше чуть том нельзя такой им более "
               "всегда конечно всю между".split())
_WORD = re.compile(r"[^\W\d_]+", re.UNICODE)
_CYR = re.compile(r"[\u0400-\u04FF]")
_LAT = re.compile(r"[A-Za-z]")

CJK_PATTERN = re.compile(r"[\u4e00-\u9fff\u3040-\u30ff\u3400-\u4dbf\uff00-\uffef\uac00-\ud7af\u1100-\u11ff]")


def language_scores(text: str) -> dict:
    words = [w.lower() for w in _WORD.findall(text or "")]
    cyr = len(_CYR.findall(text or ""))
    lat = len(_LAT.findall(text or ""))
    letters = cyr + lat
    s_en = s_ru = 0.0
    if letters:
        s_en += 2.0 * lat / letters
        s_ru += 2.0 * cyr / letters
    if words:
        s_en += sum(w in _EN_STOP for w in words) / len(words)
        s_ru += sum(w in _RU_STOP for w in words) / len(words)
    return {"en": s_en, "ru": s_ru}


def get_language(text: str) -> str:
    """'en' or 'ru' (ties / empty text resolve to 'en', as langid does on empty input)."""
    s = language_scores(text)
    lang = "ru" if s["ru"] > s["en"] else "en"
    logger.debug("detected language %s %s for %r", lang, s, (text or "")[:100])
    return lang


def has_cjk_characters(text: str) -> bool:
    return bool(CJK_PATTERN.search(text or ""))
