"""LLM Markdown -> Telegram MarkdownV2 (reference bot/platforms/telegram/format.py).

The reference converts Markdown to HTML with markdown2, walks it with BeautifulSoup and re-emits
MarkdownV2.  This module parses the Markdown subset LLMs produce directly (no markdown2 / bs4 / lxml):

  blocks : paragraphs, ATX headings (-> bold paragraph), fenced code (```lang), bullet lists
           (-, *, +) and ordered lists (1.) with nesting by indentation, block quotes (>)
  inline : `code`, **bold** / __bold__, *italic* / _italic_, ***bold italic***, ~~strike~~,
           [text](url)

Everything outside entities is escaped with MarkdownV2's rules (code keeps only ` and \\ escaped,
link targets only ) and \\).  Blocks are separated by a blank line, list items by a newline.  Any
parser error falls back to fully escaped text, so a message can always be sent.
"""
from __future__ import annotations

import logging
import re

logger = logging.getLogger(__name__)

_SPECIAL = re.compile(r"([_*\[\]()~`>#+\-=|{}.!\\])")
_SPECIAL_NO_QUOTE = re.compile(r"([_*\[\]()~>#+\-=|{}.!\\])")


def escape_markdownV2(text: str) -> str:
    """Escape every MarkdownV2 special character except the backquote."""
    return _SPECIAL_NO_QUOTE.sub(r"\\\1", text)


def escape_markdownV2_with_quote(text: str) -> str:
    return _SPECIAL.sub(r"\\\1", text)


def _escape_code(text: str) -> str:
    return text.replace("\\", "\\\\").replace("`", "\\`")


def _escape_url(url: str) -> str:
    return url.replace("\\", "\\\\").replace(")", "\\)")


# ------------------------------------------------------------------------------------------ inline

_INLINE = re.compile(
    r"(?P<code>(?<!\\)`(?P<code_body>[^`\n]+)`)"
    r"|(?P<link>\[(?P<link_text>[^\]\n]+)\]\((?P<link_url>[^)\s]+)\))"
    r"|(?P<bi>\*\*\*(?P<bi_body>.+?)\*\*\*)"
    r"|(?P<b>\*\*(?P<b_body>.+?)\*\*|__(?P<b2_body>.+?)__)"
    r"|(?P<s>~~(?P<s_body>.+?)~~)"
    r"|(?P<i>(?<![\w*])\*(?P<i_body>[^*\s](?:[^*]*[^*\s])?)\*(?![\w*])|(?<!\w)_(?P<i2_body>[^_\s](?:[^_]*[^_\s])?)_(?!\w))",
    re.S,
)


def format_inline(text: str) -> str:
    out, pos = [], 0
    for m in _INLINE.finditer(text):
        out.append(escape_markdownV2_with_quote(text[pos:m.start()]))
        if m.group("code"):
            out.append(f"`{_escape_code(m.group('code_body'))}`")
        elif m.group("link"):
            out.append(f"[{format_inline(m.group('link_text'))}]({_escape_url(m.group('link_url'))})")
        elif m.group("bi"):
            out.append(f"*{format_inline(m.group('bi_body'))}*")
        elif m.group("b"):
            out.append(f"*{format_inline(m.group('b_body') or m.group('b2_body'))}*")
        elif m.group("s"):
            out.append(f"~{format_inline(m.group('s_body'))}~")
        elif m.group("i"):
            out.append(f"_{format_inline(m.group('i_body') or m.group('i2_body'))}_")
        pos = m.end()
    out.append(escape_markdownV2_with_quote(text[pos:]))
    return "".join(out)


# ------------------------------------------------------------------------------------------ blocks

_FENCE = re.compile(r"^\s*```")
_HEADING = re.compile(r"^\s{0,3}(#{1,6})\s+(.*?)\s*#*\s*$")
_BULLET = re.compile(r"^(\s*)([-*+])\s+(.*)$")
_ORDERED = re.compile(r"^(\s*)(\d{1,9})[.)]\s+(.*)$")
_QUOTE = re.compile(r"^\s*>\s?(.*)$")


def _blocks(lines):
    """Yield ('code', text) | ('heading', text) | ('list', [(indent, marker, text)]) |
    ('quote', [lines]) | ('para', [lines])."""
    i, n = 0, len(lines)
    while i < n:
        line = lines[i]
        if not line.strip():
            i += 1
            continue
        if _FENCE.match(line):
            body = []
            i += 1
            while i < n and not _FENCE.match(lines[i]):
                body.append(lines[i])
                i += 1
            i += 1  # closing fence (or EOF)
            yield "code", "\n".join(body)
            continue
        m = _HEADING.match(line)
        if m:
            yield "heading", m.group(2)
            i += 1
            continue
        if _BULLET.match(line) or _ORDERED.match(line):
            items = []
            while i < n and lines[i].strip():
                mb, mo = _BULLET.match(lines[i]), _ORDERED.match(lines[i])
                if mb:
                    items.append([len(mb.group(1).expandtabs(4)), None, mb.group(3)])
                elif mo:
                    items.append([len(mo.group(1).expandtabs(4)), int(mo.group(2)), mo.group(3)])
                elif items:  # lazy continuation line
                    items[-1][2] += " " + lines[i].strip()
                i += 1
            yield "list", items
            continue
        if _QUOTE.match(line):
            q = []
            while i < n and _QUOTE.match(lines[i]):
                q.append(_QUOTE.match(lines[i]).group(1))
                i += 1
            yield "quote", q
            continue
        para = []
        while i < n and lines[i].strip() and not (_FENCE.match(lines[i]) or _HEADING.match(lines[i])
                                                  or _BULLET.match(lines[i]) or _ORDERED.match(lines[i])
                                                  or _QUOTE.match(lines[i])):
            para.append(lines[i].strip())
            i += 1
        yield "para", para


def _format_list(items) -> str:
    levels: list = []
    out = []
    for indent, number, text in items:
        while levels and indent < levels[-1]:
            levels.pop()
        if not levels or indent > levels[-1]:
            levels.append(indent)
        depth = len(levels) - 1
        marker = "\\-" if number is None else f"{number}\\."
        out.append(f"{'  ' * depth}{marker} {format_inline(text)}")
    return "\n".join(out)


def format_markdownV2(text: str) -> str:
    try:
        parts = []
        for kind, body in _blocks((text or "").replace("\r\n", "\n").split("\n")):
            if kind == "code":
                parts.append(f"```\n{_escape_code(body)}\n```")
            elif kind == "heading":
                parts.append(f"*{format_inline(body)}*")
            elif kind == "list":
                parts.append(_format_list(body))
            elif kind == "quote":
                parts.append("\n".join(f">{format_inline(q)}" for q in body))
            else:
                parts.append("\n".join(format_inline(line) for line in body))
        return "\n\n".join(parts)
    except Exception:  # pragma: no cover - defensive: never fail a delivery on formatting
        logger.exception("MarkdownV2 formatting failed")
        return escape_markdownV2_with_quote(text or "")


class TelegramMarkdownV2FormattedText(str):
    """A ``str`` holding the MarkdownV2 rendering; ``raw_text`` keeps the source."""

    raw_text: str

    def __new__(cls, text: str):
        obj = str.__new__(cls, format_markdownV2(text))
        obj.raw_text = text
        return obj
