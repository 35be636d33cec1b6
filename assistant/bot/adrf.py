"""Async dispatch for DRF views (reference bot/adrf.py): DRF's ``APIView.dispatch`` is synchronous;
this mixin awaits coroutine handlers and runs sync ones (and DRF's ``initial`` checks) in a thread."""
import asyncio

from assistant.utils.sync import sync_to_async


class AsyncMixin:
    """Must come first in the bases: ``class V(AsyncMixin, APIView)``."""

    @classmethod
    def as_view(cls, *args, **initkwargs):
        view = super().as_view(*args, **initkwargs)

        async def async_view(*a, **kw):
            return await view(*a, **kw)

        async_view.csrf_exempt = True
        return async_view

    async def dispatch(self, request, *args, **kwargs):
        self.args, self.kwargs = args, kwargs
        request = self.initialize_request(request, *args, **kwargs)
        self.request = request
        self.headers = self.default_response_headers
        try:
            await sync_to_async(self.initial)(request, *args, **kwargs)
            name = request.method.lower()
            handler = getattr(self, name, self.http_method_not_allowed) if name in self.http_method_names \
                else self.http_method_not_allowed
            if not asyncio.iscoroutinefunction(handler):
                handler = sync_to_async(handler)
            response = await handler(request, *args, **kwargs)
        except Exception as exc:
            response = self.handle_exception(exc)
        self.response = self.finalize_response(request, response, *args, **kwargs)
        return self.response
