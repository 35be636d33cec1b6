"""Tiny async JSON-over-HTTP client shared by the remote providers (aiohttp, no vendor SDKs)."""
from __future__ import annotations

import json
from typing import Any

import aiohttp


class HTTPError(Exception):
    def __init__(self, status: int, body: str, url: str):
        super().__init__(f"HTTP {status} from {url}: {body[:500]}")
        self.status, self.body, self.url = status, body, url


async def post_json(url: str, payload: dict, headers: dict | None = None, timeout: float = 300.0) -> Any:
    to = aiohttp.ClientTimeout(total=timeout)
    async with aiohttp.ClientSession(timeout=to) as session:
        async with session.post(url, json=payload, headers=headers or {}) as resp:
            text = await resp.text()
            if resp.status != 200:
                raise HTTPError(resp.status, text, url)
            return json.loads(text) if text else None
