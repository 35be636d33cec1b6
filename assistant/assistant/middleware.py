"""Absolute MEDIA_URL (reference assistant/assistant/middleware.py).  Telegram and API clients need
absolute photo URLs; the first request's scheme+host is used (the reference re-derived it on every
request but, because it mutated settings, also kept the first one)."""
import threading

from django.conf import settings

_lock = threading.Lock()


class MediaURLMiddleware:
    def __init__(self, get_response):
        self.get_response = get_response

    def __call__(self, request):
        if not settings.MEDIA_URL.startswith("http"):
            with _lock:
                if not settings.MEDIA_URL.startswith("http"):
                    scheme = "https" if request.is_secure() else "http"
                    settings.MEDIA_URL = f"{scheme}://{request.get_host()}{settings.MEDIA_URL}"
        return self.get_response(request)
