"""CSV knowledge-base loader (reference loading/csv.py:14-53).

The file has a header row and three columns ``(toc_title, doc_name, doc_content)``: every row becomes a
child ``WikiDocument`` under a root page per TOC title (created on first use), all in one transaction;
each saved page then triggers ingest (assistant.processing.signals).  ``read_rows`` is the Django-free
parser (UTF-8 with or without BOM; titles whitespace-normalised; rows of the wrong width are an
error naming the line)."""
from __future__ import annotations

import csv
import logging
import re
from typing import Iterator, Tuple

logger = logging.getLogger(__name__)

COLUMNS_COUNT = 3


def normalize_title(name: str) -> str:
    return re.sub(r"\s+", " ", name or "").strip()


def read_rows(path: str) -> Iterator[Tuple[str, str, str]]:
    with open(path, newline="", encoding="utf-8-sig") as f:
        reader = csv.reader(f)
        header = next(reader, None)
        if header is None:
            return
        if len(header) != COLUMNS_COUNT:
            raise ValueError(f"expected {COLUMNS_COUNT} columns, header has {len(header)}")
        for line, row in enumerate(reader, start=2):
            if not any(c.strip() for c in row):
                continue
            if len(row) != COLUMNS_COUNT:
                raise ValueError(f"line {line}: expected {COLUMNS_COUNT} columns, got {len(row)}")
            toc, name, content = row
            yield normalize_title(toc), normalize_title(name), content.strip()


class CSVLoader:
    def __init__(self, bot, filepath: str):
        self._bot = bot
        self._filepath = filepath

    async def load(self) -> int:
        from assistant.utils.sync import sync_to_async
        return await sync_to_async(self.load_sync)()

    def load_sync(self) -> int:
        from django.db import transaction

        from assistant.storage.models import WikiDocument

        n = 0
        with transaction.atomic():
            roots = {}
            for toc, name, content in read_rows(self._filepath):
                parent = roots.get(toc)
                if parent is None:
                    parent, _ = WikiDocument.objects.get_or_create(bot=self._bot, title=toc, parent=None)
                    roots[toc] = parent
                WikiDocument.objects.create(bot=self._bot, title=name, content=content, parent=parent)
                n += 1
        logger.info("loaded %d wiki documents from %s", n, self._filepath)
        return n
